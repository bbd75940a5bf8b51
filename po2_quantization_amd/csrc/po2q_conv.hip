// Convolution kernels for gfx950 (QuantizedConv2d.forward, models/quantized_conv.py:32-38,
// i.e. F.conv2d(x, Q(w), bias, stride, padding, dilation, groups), NCHW fp32).
//
// kind 0  conv_mfma_f32: LDS-staged implicit GEMM on v_mfma_f32_16x16x4_f32.
//         D[out-channel][pixel] += W[out-channel][c..c+3 @ tap] * X[c..c+3 @ tap][pixel]
//         Block = 4 waves; tile = 16*MI output channels x TP*TQ output pixels of
//         one image; each wave owns NJ groups of 16 pixels.  Per input-channel
//         chunk the halo tile [CC][HH][WW] (fp32, NCHW order, zero padded) and
//         the chunk's packed weights are staged in LDS; fragments are read with
//         conflict-free ds_read_b32 (pixels on lanes, channels on lane>>4).
// kind 1  conv_depthwise: direct conv, one output pixel per lane (HBM-bound).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <array>
#include <cstdlib>
#include <map>
#include <mutex>

#include "po2q_epi.h"
#include "po2q_internal.h"

namespace po2q {

typedef float floatx4 __attribute__((ext_vector_type(4)));

struct ConvArgs {
    int N, C, H, W, K, R, S, sh, sw, ph, pw, dh, dw, groups;
    int P, Q, Cg, Kg;
    int TP, TQ, tilesP, tilesQ, CC, nchunks, kblocks;
    int HH, WW, WWp, PS, steps;
};

static ConvArgs to_args(const ConvPlan& p) {
    ConvArgs a;
    a.N = p.N; a.C = p.C; a.H = p.H; a.W = p.W; a.K = p.K; a.R = p.R; a.S = p.S;
    a.sh = p.sh; a.sw = p.sw; a.ph = p.ph; a.pw = p.pw; a.dh = p.dh; a.dw = p.dw; a.groups = p.groups;
    a.P = p.P; a.Q = p.Q; a.Cg = p.Cg; a.Kg = p.Kg;
    a.TP = p.TP; a.TQ = p.TQ; a.tilesP = p.tilesP; a.tilesQ = p.tilesQ; a.CC = p.CC;
    a.nchunks = p.nchunks; a.kblocks = p.kblocks;
    a.HH = p.HH; a.WW = p.WW; a.WWp = p.WWp; a.PS = p.PS; a.steps = p.steps;
    return a;
}

template <int MI, int NJ>
__global__ __launch_bounds__(kThreads) void conv_mfma_f32(const float* __restrict__ x,
                                                          const float* __restrict__ wpk,
                                                          const float* __restrict__ bias,
                                                          float* __restrict__ y, ConvArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* xs = smem;                  // [CC][PS]  halo tile, plane stride PS, row stride WWp
    float* wsm = smem + a.CC * a.PS;   // [steps][MI][64] packed weights of the chunk

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int bid = blockIdx.x;
    const int tiles = a.tilesP * a.tilesQ;
    const int tile = bid % tiles; bid /= tiles;
    const int kb = bid % a.kblocks; bid /= a.kblocks;
    const int g = bid % a.groups;
    const int n = bid / a.groups;
    const int p0 = (tile / a.tilesQ) * a.TP, q0 = (tile % a.tilesQ) * a.TQ;
    const int h0 = p0 * a.sh - a.ph, w0 = q0 * a.sw - a.pw;
    const int npix = a.TP * a.TQ;

    int poff[NJ];
#pragma unroll
    for (int nj = 0; nj < NJ; ++nj) {
        int slot = (wave * NJ + nj) * 16 + (lane & 15);
        if (slot >= npix) slot = 0;
        const int pl = slot / a.TQ, ql = slot - pl * a.TQ;
        poff[nj] = pl * a.sh * a.WWp + ql * a.sw + (lane >> 4) * a.PS;
    }

    floatx4 acc[MI][NJ];
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int nj = 0; nj < NJ; ++nj) acc[mi][nj] = floatx4{0.f, 0.f, 0.f, 0.f};

    const int chunk_floats = a.steps * MI * 64;
    const float* wsrc = wpk + (int64_t)(g * a.kblocks + kb) * a.nchunks * chunk_floats;
    const int c4n = a.CC >> 2;

    for (int chunk = 0; chunk < a.nchunks; ++chunk) {
        const int c0 = chunk * a.CC;
        // ---- stage halo tile: one (channel, row) per wave iteration, lanes along W
        const float* xg = x + ((int64_t)n * a.C + (int64_t)g * a.Cg + c0) * a.H * a.W;
        const int rows = a.CC * a.HH;
        for (int row = wave; row < rows; row += 4) {
            const int c = row / a.HH, hh = row - c * a.HH;
            const int h = h0 + hh;
            const bool rv = (c0 + c < a.Cg) && (h >= 0) && (h < a.H);
            const float* src = xg + ((int64_t)c * a.H + h) * a.W;
            float* dst = xs + c * a.PS + hh * a.WWp;
            for (int ww = lane; ww < a.WW; ww += 64) {
                const int w = w0 + ww;
                dst[ww] = (rv && w >= 0 && w < a.W) ? src[w] : 0.0f;
            }
        }
        // ---- stage packed weights (contiguous, float4)
        const float4* ws4 = reinterpret_cast<const float4*>(wsrc + (int64_t)chunk * chunk_floats);
        float4* wd4 = reinterpret_cast<float4*>(wsm);
        for (int e = tid; e < (chunk_floats >> 2); e += kThreads) wd4[e] = ws4[e];
        __syncthreads();

        for (int r = 0; r < a.R; ++r) {
            for (int s = 0; s < a.S; ++s) {
                const int tap = r * a.dh * a.WWp + s * a.dw;
                const int tbase = (r * a.S + s) * c4n;
                for (int c4 = 0; c4 < c4n; ++c4) {
                    const float* wrow = wsm + (tbase + c4) * MI * 64 + lane;
                    float av[MI], bv[NJ];
#pragma unroll
                    for (int mi = 0; mi < MI; ++mi) av[mi] = wrow[mi * 64];
                    const float* xrow = xs + c4 * 4 * a.PS + tap;
#pragma unroll
                    for (int nj = 0; nj < NJ; ++nj) bv[nj] = xrow[poff[nj]];
#pragma unroll
                    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
                        for (int nj = 0; nj < NJ; ++nj)
                            acc[mi][nj] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[mi], bv[nj], acc[mi][nj], 0, 0, 0);
                }
            }
        }
        __syncthreads();
    }

    // ---- epilogue: D[row = 4*(lane>>4)+i][col = lane&15] -> y[n][k][p][q]
#pragma unroll
    for (int nj = 0; nj < NJ; ++nj) {
        const int slot = (wave * NJ + nj) * 16 + (lane & 15);
        if (slot >= npix) continue;
        const int pl = slot / a.TQ, ql = slot - pl * a.TQ;
        const int pp = p0 + pl, qq = q0 + ql;
        if (pp >= a.P || qq >= a.Q) continue;
#pragma unroll
        for (int mi = 0; mi < MI; ++mi) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int kk = kb * MI * 16 + mi * 16 + 4 * (lane >> 4) + i;
                if (kk >= a.Kg) continue;
                const int k = g * a.Kg + kk;
                float v = acc[mi][nj][i];
                if (bias) v += bias[k];
                y[(((int64_t)n * a.K + k) * a.P + pp) * a.Q + qq] = v;
            }
        }
    }
}

// Depthwise (groups == C, K = groups * Kg): one output element per lane.
// EPI: the eval epilogue in the store, y = act((acc + bias) * ps[k] + pb[k] + res) (ps / pb / res
// optional) -- the fused entry's semantics, so a depthwise layer this kernel takes (small spatial
// sizes) needs no second elementwise pass.
template <bool EPI>
__global__ __launch_bounds__(kThreads) void conv_depthwise(const float* __restrict__ x, const float* __restrict__ qw,
                                                           const float* __restrict__ bias, float* __restrict__ y,
                                                           ConvArgs a, const float* __restrict__ ps,
                                                           const float* __restrict__ pb, const float* __restrict__ res,
                                                           int act) {
    const int64_t total = (int64_t)a.N * a.K * a.P * a.Q;
    const int64_t stride = (int64_t)gridDim.x * kThreads;
    for (int64_t idx = (int64_t)blockIdx.x * kThreads + threadIdx.x; idx < total; idx += stride) {
        int64_t t = idx;
        const int q = (int)(t % a.Q); t /= a.Q;
        const int p = (int)(t % a.P); t /= a.P;
        const int k = (int)(t % a.K);
        const int n = (int)(t / a.K);
        const int c = k / a.Kg;  // Cg == 1
        const float* xc = x + ((int64_t)n * a.C + c) * a.H * a.W;
        const float* wk = qw + (int64_t)k * a.R * a.S;
        float acc = 0.0f;
        for (int r = 0; r < a.R; ++r) {
            const int h = p * a.sh - a.ph + r * a.dh;
            if (h < 0 || h >= a.H) continue;
            for (int s = 0; s < a.S; ++s) {
                const int w = q * a.sw - a.pw + s * a.dw;
                if (w < 0 || w >= a.W) continue;
                acc = fmaf(xc[(int64_t)h * a.W + w], wk[r * a.S + s], acc);
            }
        }
        if (bias) acc += bias[k];
        if constexpr (EPI) {
            if (ps) acc *= ps[k];
            if (pb) acc += pb[k];
            if (res) acc += res[idx];
            acc = epi_act(acc, act);
        }
        y[idx] = acc;
    }
}

hipError_t launch_conv_depthwise_epi(const ConvPlan& p, const float* x, const float* packed, const float* bias, float* y,
                                     const float* ps, const float* pb, const float* res, int act, hipStream_t s) {
    hipLaunchKernelGGL(conv_depthwise<true>, dim3((unsigned)p.blocks), dim3(kThreads), 0, s, x, packed, bias, y,
                       to_args(p), ps, pb, res, act);
    return hipGetLastError();
}

// ------------------------------------------------------------------ planning --
static int ceil_div(int a, int b) { return (a + b - 1) / b; }

// Geometry validation (the reference's F.conv2d error conditions) and derived sizes.
static bool plan_geometry(ConvPlan& p, int64_t N, int64_t C, int64_t H, int64_t W, int64_t K, int64_t R,
                          int64_t S, int64_t sh, int64_t sw, int64_t ph, int64_t pw, int64_t dh, int64_t dw,
                          int64_t groups) {
    if (N <= 0 || C <= 0 || H <= 0 || W <= 0 || K <= 0 || R <= 0 || S <= 0 || groups <= 0) {
        set_error("po2q: all sizes must be positive");
        return false;
    }
    if (sh <= 0 || sw <= 0 || dh <= 0 || dw <= 0 || ph < 0 || pw < 0) {
        set_error("po2q: stride/dilation must be positive and padding non-negative");
        return false;
    }
    if (C % groups != 0 || K % groups != 0) {
        set_error("po2q: in_channels and out_channels must be divisible by groups");
        return false;
    }
    const int64_t P = (H + 2 * ph - dh * (R - 1) - 1) / sh + 1;
    const int64_t Q = (W + 2 * pw - dw * (S - 1) - 1) / sw + 1;
    if (H + 2 * ph < dh * (R - 1) + 1 || W + 2 * pw < dw * (S - 1) + 1 || P <= 0 || Q <= 0) {
        set_error("po2q: kernel size can't be greater than actual (padded) input size");
        return false;
    }
    const int64_t lim = INT_MAX;
    if (N * C > lim || N * K > lim || H * W > lim || P * Q > lim || K * (C / groups) * R * S > lim ||
        C * H * W > lim || K * P * Q > lim) {
        set_error("po2q: tensor too large for 32-bit per-image indexing");
        return false;
    }
    p.N = (int)N; p.C = (int)C; p.H = (int)H; p.W = (int)W; p.K = (int)K; p.R = (int)R; p.S = (int)S;
    p.sh = (int)sh; p.sw = (int)sw; p.ph = (int)ph; p.pw = (int)pw; p.dh = (int)dh; p.dw = (int)dw;
    p.groups = (int)groups; p.P = (int)P; p.Q = (int)Q; p.Cg = (int)(C / groups); p.Kg = (int)(K / groups);

    p.NT = 0; p.SB = 0; p.plane = 0; p.taps = p.R * p.S; p.vrx = 0;
    p.dma_d0 = p.dma_nck = p.dma_ni = p.dma_nw = 0; p.dma_waves = 0; p.dma_ov = 0; p.pd = 0; p.nts = 0; p.fp = 0;
    return true;
}

static bool bf16x3_wanted(const ConvPlan& p, int mode, int flags) {
    return flags == 2 || (flags == 0 && mode != 0 && !(p.Cg == 1 && p.groups > 1));
}

// Any PO2Q_* tile/kernel tuning knob set: the planners obey it and the autotune cache is bypassed.
static bool tuning_knobs() {
    return getenv("PO2Q_X3_TILE") || getenv("PO2Q_X3P_TILE") || getenv("PO2Q_X3P_WAVES") || getenv("PO2Q_NO_DMA");
}

// Heuristic kernel choice between the two bf16x3 kernels, from the per-layer sweeps
// (profiles/r01_v3_tile_sweep.jsonl): the LDS-DMA kernel wins on stride-2 3x3 layers
// and on 3x3 stride-1 layers with 17..32 output channels, the register-staged kernel
// elsewhere.  po2q_qconv2d_autotune replaces this with a measurement.
static bool prefer_dma(const ConvPlan& p) {
    if (getenv("PO2Q_X3P_TILE") || getenv("PO2Q_X3P_WAVES")) return true;
    if (getenv("PO2Q_X3_TILE")) return false;
    if (p.R == 3 && p.S == 3 && p.sh == 2 && p.sw == 2) return true;
    return p.R == 3 && p.S == 3 && p.sh == 1 && p.sw == 1 && p.K > 16 && p.K <= 32;
}

// ------------------------------------------------------------ autotune cache --
using PlanKey = std::array<int64_t, 18>;
static std::mutex g_tuned_mu;
static std::map<PlanKey, ConvPlan> g_tuned;

static PlanKey plan_key(const ConvPlan& p, int mode, int bits, int fsr, int flags) {
    return {p.N, p.C, p.H, p.W, p.K, p.R, p.S, p.sh, p.sw, p.ph, p.pw, p.dh, p.dw, p.groups, mode, bits, fsr, flags};
}

void tuned_store(const ConvPlan& p, int mode, int bits, int fsr, int flags) {
    std::lock_guard<std::mutex> g(g_tuned_mu);
    g_tuned[plan_key(p, mode, bits, fsr, flags)] = p;
}

static bool tuned_lookup(ConvPlan& p, int mode, int bits, int fsr, int flags) {
    std::lock_guard<std::mutex> g(g_tuned_mu);
    auto it = g_tuned.find(plan_key(p, mode, bits, fsr, flags));
    if (it == g_tuned.end()) return false;
    p = it->second;
    return true;
}

static bool plan_fallback(ConvPlan& p, bool dw3 = true);

// Heuristic plan + the ranked bf16x3 alternatives (empty unless bf16x3 applies).
static bool plan_heuristic(ConvPlan& p, int mode, int bits, int fsr, int flags, std::vector<PlanCand>* reg_out,
                           std::vector<PlanCand>* dma_out, std::vector<PlanCand>* rows_out = nullptr,
                           std::vector<PlanCand>* pw_out = nullptr) {
    if (mode == 0 && flags != 2) {
        // unquantized weights: the direct stem kernel / the fp32 pointwise GEMM where they apply,
        // the generic fp32 MFMA kernel as the autotuner's alternative
        std::vector<PlanCand> f32;
        f32s_candidates(p, f32);
        if (!f32.empty()) {
            std::stable_sort(f32.begin(), f32.end(), [](const PlanCand& u, const PlanCand& v) { return u.cost < v.cost; });
            PlanCand fb{1e30, p};
            const bool fb_ok = plan_fallback(fb.plan);
            if (fb_ok) f32.push_back(fb);
            p = f32[0].plan;
            if (pw_out) *pw_out = std::move(f32);
            return true;
        }
    }
    if (bf16x3_wanted(p, mode, flags)) {
        std::vector<PlanCand> reg, dma;
        x3_candidates(p, mode, bits, fsr, reg);
        if (!reg.empty()) {
            const char* nd = getenv("PO2Q_NO_DMA");  // A/B knob: keep the register-staged kernel
            if (!(nd && nd[0] == '1')) x3p_candidates(p, dma);
            std::vector<PlanCand> rows;
            rows_candidates(p, mode, bits, fsr, rows);
            std::stable_sort(rows.begin(), rows.end(),
                             [](const PlanCand& u, const PlanCand& v) { return u.cost < v.cost; });
            p = (!dma.empty() && prefer_dma(p)) ? dma[0].plan : reg[0].plan;
            // the row-streaming kernels beat both tile kernels on every shape they take
            // (profiles/r01_v9_plan_sweep.jsonl, r01_v10_plan_sweep.jsonl)
            if (!rows.empty() && !tuning_knobs()) p = rows[0].plan;
            // 1x1 / stride 1: the pointwise GEMM kernel (no halo, no LDS, fused epilogue)
            std::vector<PlanCand> pwc;
            pw_candidates(p, mode, bits, fsr, pwc);
            if (!pwc.empty() && !tuning_knobs()) p = pwc[0].plan;
            // small images (CIFAR sizes): the LDS-resident block kernel; its candidates ride on
            // the pointwise list (the two never apply to the same shape)
            if (pwc.empty()) {
                img_candidates(p, mode, bits, fsr, pwc);
                if (!pwc.empty() && p.W <= 32 && !tuning_knobs()) p = pwc[0].plan;
            }
            if (pw_out) *pw_out = std::move(pwc);
            if (rows_out) *rows_out = std::move(rows);
            if (reg_out) *reg_out = std::move(reg);
            if (dma_out) *dma_out = std::move(dma);
            return true;
        }
        if (flags == 2) {
            set_error("po2q: bf16x3 precision needs power-of-two weights (mode po2/po2+, exponents within the "
                      "bf16 range) and groups == 1");
            return false;
        }
    }
    return plan_fallback(p);
}

bool plan_candidates(std::vector<ConvPlan>& out, int64_t N, int64_t C, int64_t H, int64_t W, int64_t K, int64_t R,
                     int64_t S, int64_t sh, int64_t sw, int64_t ph, int64_t pw, int64_t dh, int64_t dw,
                     int64_t groups, int mode, int bits, int fsr, int flags);

bool make_plan(ConvPlan& p, int64_t N, int64_t C, int64_t H, int64_t W, int64_t K, int64_t R, int64_t S,
               int64_t sh, int64_t sw, int64_t ph, int64_t pw, int64_t dh, int64_t dw, int64_t groups, int mode,
               int bits, int fsr, int flags) {
    if (!plan_geometry(p, N, C, H, W, K, R, S, sh, sw, ph, pw, dh, dw, groups)) return false;
    if (const char* force = getenv("PO2Q_PLAN")) {  // test / tuning knob: candidate index for every call
        std::vector<ConvPlan> cands;
        const int idx = atoi(force);
        if (plan_candidates(cands, N, C, H, W, K, R, S, sh, sw, ph, pw, dh, dw, groups, mode, bits, fsr, flags) &&
            idx >= 0 && idx < (int)cands.size()) {
            p = cands[idx];
            return true;
        }
    }
    if (!tuning_knobs() && tuned_lookup(p, mode, bits, fsr, flags)) return true;
    return plan_heuristic(p, mode, bits, fsr, flags, nullptr, nullptr);
}

constexpr int kTuneRegCands = 6, kTuneDmaCands = 12, kTuneRowsCands = 40;

bool plan_candidates(std::vector<ConvPlan>& out, int64_t N, int64_t C, int64_t H, int64_t W, int64_t K, int64_t R,
                     int64_t S, int64_t sh, int64_t sw, int64_t ph, int64_t pw, int64_t dh, int64_t dw,
                     int64_t groups, int mode, int bits, int fsr, int flags) {
    ConvPlan p;
    if (!plan_geometry(p, N, C, H, W, K, R, S, sh, sw, ph, pw, dh, dw, groups)) return false;
    std::vector<PlanCand> reg, dma, rows, pwc;
    if (!plan_heuristic(p, mode, bits, fsr, flags, &reg, &dma, &rows, &pwc)) return false;
    out.clear();
    out.push_back(p);
    if (p.kind == KIND_DEPTHWISE && p.vrx == 1) {  // the one-output-per-lane kernel as the alternative
        ConvPlan l;
        const bool ok = plan_geometry(l, N, C, H, W, K, R, S, sh, sw, ph, pw, dh, dw, groups) &&
                        plan_fallback(l, false);
        if (ok && l.vrx == 0) out.push_back(l);
    }
    auto add = [&](const std::vector<PlanCand>& v, int n) {
        for (int i = 0; i < (int)v.size() && i < n; ++i) {
            const ConvPlan& c = v[i].plan;
            bool dup = false;
            for (const ConvPlan& o : out)
                dup |= o.kind == c.kind && o.NJ == c.NJ && o.MI == c.MI && o.TP == c.TP && o.TQ == c.TQ && o.vrx == c.vrx &&
                       o.dma_waves == c.dma_waves && o.dma_ov == c.dma_ov &&
                       o.dma_nw == c.dma_nw && o.pd == c.pd && o.nts == c.nts && o.PS == c.PS && o.fp == c.fp &&
                       (c.kind != KIND_BF16X3_IMG || o.kblocks == c.kblocks);
            if (!dup) out.push_back(c);
        }
    };
    add(pwc, 12);
    add(rows, kTuneRowsCands);
    add(reg, kTuneRegCands);
    add(dma, kTuneDmaCands);
    return true;
}

static bool plan_fallback(ConvPlan& p, bool dw3) {
    const int N = p.N, K = p.K, R = p.R, S = p.S, P = p.P, Q = p.Q, groups = p.groups;
    if (p.Cg == 1 && groups > 1) {  // depthwise
        const char* legacy = getenv("PO2Q_DW_LEGACY");
        if (dw3 && !(legacy && legacy[0] == '1') && dw3_plan(p)) return true;
        p.kind = KIND_DEPTHWISE;
        p.vrx = 0;
        p.MI = p.NJ = 1;
        p.TP = p.TQ = p.tilesP = p.tilesQ = 1;
        p.CC = 1; p.nchunks = 1; p.kblocks = 1;
        p.HH = p.WW = p.WWp = p.PS = 0; p.steps = 0;
        p.packed_floats = (int64_t)K * R * S;
        p.lds_bytes = 0;
        int64_t total = (int64_t)N * K * P * Q;
        int64_t b = (total + kThreads - 1) / kThreads;
        p.blocks = std::min<int64_t>(std::max<int64_t>(b, 1), 65536);
        return true;
    }

    p.kind = KIND_MFMA_F32;
    p.MI = p.Kg <= 16 ? 1 : (p.Kg <= 32 ? 2 : 4);
    p.kblocks = ceil_div(p.Kg, 16 * p.MI);
    // pixel tile: NJ groups of 16 pixels per wave
    const int pix_img = p.P * p.Q;
    p.NJ = pix_img >= 256 ? 4 : (pix_img >= 128 ? 2 : 1);
    const int slots = 64 * p.NJ;
    // choose TQ among candidates minimising launched slots x halo overhead
    const int cands[] = {p.Q, 64, 56, 32, 28, 16, 8};
    double best = 1e300;
    for (int tq : cands) {
        if (tq <= 0 || tq > p.Q || tq > slots) continue;
        int tp = std::max(1, std::min(p.P, slots / tq));
        const int tilesQ = ceil_div(p.Q, tq), tilesP = ceil_div(p.P, tp);
        const double launched = (double)tilesQ * tilesP * slots;
        const int hh = (tp - 1) * p.sh + (p.R - 1) * p.dh + 1;
        const int ww = (tq - 1) * p.sw + (p.S - 1) * p.dw + 1;
        const double halo = (double)tilesQ * tilesP * hh * ww;
        const double cost = launched * 1.0 + halo * 0.5 * p.R * p.S / 9.0;
        if (cost < best) { best = cost; p.TQ = tq; p.TP = tp; }
    }
    p.tilesQ = ceil_div(p.Q, p.TQ);
    p.tilesP = ceil_div(p.P, p.TP);
    p.HH = (p.TP - 1) * p.sh + (p.R - 1) * p.dh + 1;
    p.WW = (p.TQ - 1) * p.sw + (p.S - 1) * p.dw + 1;
    p.WWp = p.WW;
    const int plane = p.HH * p.WWp;
    // plane stride: lanes 16..31 read channel +1; offset it by 16 banks (stride 1)
    // or 1 bank (stride 2: lanes already spread over even banks)
    const int want = (p.sw == 1) ? 16 : 1;
    p.PS = plane + ((want - plane % 32) + 32) % 32;
    // channel chunk: multiple of 4, LDS <= 64 KiB
    const int cg4 = ceil_div(p.Cg, 4) * 4;
    int cc = std::min(cg4, 64);
    auto lds_for = [&](int c) {
        return (size_t)(c * p.PS + p.R * p.S * (c / 4) * p.MI * 64) * sizeof(float);
    };
    while (cc > 4 && lds_for(cc) > 64 * 1024) cc -= 4;
    if (lds_for(cc) > 64 * 1024) {
        set_error("po2q: conv tile does not fit in LDS (kernel too large)");
        return false;
    }
    p.CC = cc;
    p.nchunks = ceil_div(p.Cg, cc);
    p.steps = p.R * p.S * (cc / 4);
    p.lds_bytes = lds_for(cc);
    p.packed_floats = (int64_t)groups * p.kblocks * p.nchunks * p.steps * p.MI * 64;
    p.blocks = (int64_t)N * groups * p.kblocks * p.tilesP * p.tilesQ;
    if (p.blocks > INT_MAX) {
        set_error("po2q: grid too large");
        return false;
    }
    return true;
}

template <int MI, int NJ>
static hipError_t launch_mfma(const ConvPlan& p, const float* x, const float* packed, const float* bias, float* y,
                              hipStream_t s) {
    hipLaunchKernelGGL((conv_mfma_f32<MI, NJ>), dim3((unsigned)p.blocks), dim3(kThreads), p.lds_bytes, s, x, packed,
                       bias, y, to_args(p));
    return hipGetLastError();
}

template <int MI>
static hipError_t launch_mfma_nj(const ConvPlan& p, const float* x, const float* packed, const float* bias, float* y,
                                 hipStream_t s) {
    switch (p.NJ) {
        case 1: return launch_mfma<MI, 1>(p, x, packed, bias, y, s);
        case 2: return launch_mfma<MI, 2>(p, x, packed, bias, y, s);
        default: return launch_mfma<MI, 4>(p, x, packed, bias, y, s);
    }
}

hipError_t launch_conv(const ConvPlan& p, const float* x, const float* packed, const float* bias, float* y,
                       hipStream_t s) {
    if (p.kind == KIND_DEPTHWISE && p.vrx == 1)
        return launch_conv_dw3(p, x, packed, bias, y, nullptr, nullptr, nullptr, 0, s);
    if (p.kind == KIND_DEPTHWISE) {
        hipLaunchKernelGGL(conv_depthwise<false>, dim3((unsigned)p.blocks), dim3(kThreads), 0, s, x, packed, bias, y,
                           to_args(p), nullptr, nullptr, nullptr, 0);
        return hipGetLastError();
    }
    switch (p.MI) {
        case 1: return launch_mfma_nj<1>(p, x, packed, bias, y, s);
        case 2: return launch_mfma_nj<2>(p, x, packed, bias, y, s);
        default: return launch_mfma_nj<4>(p, x, packed, bias, y, s);
    }
}

}  // namespace po2q
