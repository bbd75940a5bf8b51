// bf16x3 split-exact implicit-GEMM convolution for gfx950 (the PO2 hot path).
//
// Reference: QuantizedConv2d.forward (models/quantized_conv.py:32-38) =
//   F.conv2d(x, Q(w), bias, stride, padding, dilation) with Q the PO2 / PO2+
//   quantizer (utils/quantizers.py:19-52), NCHW fp32 in and out.
//
// Why bf16 MFMA gives fp32 results here:
//   * Q(w) = (2^e * sign(w)) * scale, so W' = Q(w) / scale = +-2^e (or 0) is
//     EXACT in bf16 for every exponent the quantizer can produce (e >= -126).
//   * Every fp32 activation splits exactly into three bf16 terms by bit
//     truncation: hi = x & 0xffff0000, mid = (x - hi) & 0xffff0000,
//     lo = x - hi - mid (each remainder carries <= 16, then <= 8 significant bits).
//   * v_mfma_f32_16x16x32_bf16 forms the products W' * {hi, mid, lo} exactly and
//     accumulates in fp32; y = scale * acc (+ bias).  The only roundings are the
//     fp32 accumulations -- the same class of error as the reference's fp32 conv
//     (parity contract: max|y - y_ref| <= 1e-5 max|y_ref|, tests/_util.py).
//   Three bf16 MFMAs cost 3/16 of one fp32 MFMA (MI355X: 2.5 PF bf16 vs 157 TF
//   fp32), which moves every ResNet56 layer from the fp32 matrix roof to HBM.
//
// Kernel structure (one 256-thread block = 4 waves per output tile):
//   tile = TP x TQ output pixels of one image x (16*NT) output channels;
//   per input-channel chunk of CC channels:
//     x halo tile  HBM fp32 NCHW -> split hi/mid/lo -> LDS, three planes laid out
//                  [halo pixel][CC] bf16 (pixel stride SB = 2*CC bytes; CC = 32
//                  XOR-swizzles the channel octet with pixel bits 1..2), so an
//                  MFMA A-fragment (16 pixels x 8 consecutive k) is one
//                  conflict-free ds_read_b128 per lane (tools/lds_banks.py);
//     weights      pre-packed B fragments (po2q_quant.hip) -> LDS, 1 KiB per
//                  (k-step, 16-channel tile);
//   GEMM: M = pixels (NJ groups of 16 per wave), N = output channels (NT tiles),
//         k = (tap, channel) tap-major, 32 per MFMA k-step; padded taps read a
//         zero 16-byte slot (never a real pixel: 0 * inf must not appear).
//   Epilogue: D[pixel][channel] -> lane holds 4 consecutive pixels of one
//   channel -> one float4 store per (group, tile) into NCHW y.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdlib>

#include "po2q_internal.h"

namespace po2q {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

struct X3Args {
    int N, C, H, W, K, P, Q, sh, sw, ph, pw, dh, dw, R, S;
    int TP, TQ, tilesP, tilesQ, kblocks, nchunks, HH, WW, ksteps, taps;
    int plane;     // bytes per split plane (halo pixels * SB + 16 zero bytes)
    int w_off;     // LDS byte offset of the weight fragments
    int tap_off;   // LDS byte offset of the tap offset table
    int vec;       // float4 epilogue allowed (Q % 4 == 0 && TQ % 4 == 0)
    int remap;     // XCD-aware block remap (nblocks % 8 == 0)
    int nblocks;
};

// Exact 3-way bf16 split of 8 fp32 values (bit patterns); non-finite values keep
// their class in hi (NaN stays NaN) with mid = lo = 0.
__device__ __forceinline__ void split3(const uint32_t (&b)[8], uint4& hi, uint4& mid, uint4& lo) {
    uint32_t h16[8], m16[8], l16[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint32_t u = b[j];
        const bool nonfinite = (u & 0x7f800000u) == 0x7f800000u;
        const bool nan = nonfinite && (u & 0x007fffffu);
        const uint32_t hb = u & 0xffff0000u;
        float r1 = __uint_as_float(u) - __uint_as_float(hb);
        r1 = nonfinite ? 0.0f : r1;
        const uint32_t r1b = __float_as_uint(r1);
        const uint32_t mb = r1b & 0xffff0000u;
        const float r2 = r1 - __uint_as_float(mb);
        h16[j] = (hb >> 16) | (nan ? 0x40u : 0u);
        m16[j] = mb >> 16;
        l16[j] = __float_as_uint(r2) >> 16;
    }
    hi = make_uint4(h16[0] | (h16[1] << 16), h16[2] | (h16[3] << 16), h16[4] | (h16[5] << 16), h16[6] | (h16[7] << 16));
    mid = make_uint4(m16[0] | (m16[1] << 16), m16[2] | (m16[3] << 16), m16[4] | (m16[5] << 16), m16[6] | (m16[7] << 16));
    lo = make_uint4(l16[0] | (l16[1] << 16), l16[2] | (l16[3] << 16), l16[4] | (l16[5] << 16), l16[6] | (l16[7] << 16));
}

// LDS byte address of channel octet `coct` of halo pixel `hp` inside a plane.
template <int CC>
__device__ __forceinline__ int x_addr(int hp, int coct) {
    if constexpr (CC == 16) {
        return hp * 32 + coct * 16;
    } else {
        return hp * (2 * CC) + ((coct ^ ((hp >> 1) & 3)) << 4);
    }
}

template <int CC, int NT, int NJ>
__global__ __launch_bounds__(kThreads) void conv_bf16x3(const float* __restrict__ x, const uint4* __restrict__ wpk,
                                                        const float* __restrict__ scale_p,
                                                        const float* __restrict__ bias, float* __restrict__ y,
                                                        X3Args a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    constexpr int OCT = CC / 8;  // channel octets per tap
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

    int bid = blockIdx.x;
    if (a.remap) bid = (bid & 7) * (a.nblocks >> 3) + (bid >> 3);  // same-XCD blocks -> adjacent tiles
    const int tiles = a.tilesP * a.tilesQ;
    const int tile = bid % tiles;
    bid /= tiles;
    const int kb = bid % a.kblocks;
    const int n = bid / a.kblocks;
    const int p0 = (tile / a.tilesQ) * a.TP, q0 = (tile % a.tilesQ) * a.TQ;
    const int h0 = p0 * a.sh - a.ph, w0 = q0 * a.sw - a.pw;
    const int npix = a.TP * a.TQ;
    const int hw_halo = a.HH * a.WW;
    const int zero_off = hw_halo * (2 * CC);  // 16 zero bytes after the halo pixels of each plane

    int* tapt = reinterpret_cast<int*>(lds + a.tap_off);
    if (tid < a.taps) {
        const int r = tid / a.S, s = tid - (tid / a.S) * a.S;
        tapt[tid] = r * a.dh * a.WW + s * a.dw;
    }
    if (tid < 3) *reinterpret_cast<uint4*>(lds + tid * a.plane + zero_off) = make_uint4(0u, 0u, 0u, 0u);

    // halo pixel of this lane's pixel in each group (tile-linear, row-major)
    int hp0[NJ];
#pragma unroll
    for (int g = 0; g < NJ; ++g) {
        int slot = (wave * NJ + g) * 16 + (lane & 15);
        if (slot >= npix) slot = 0;
        const int pl = slot / a.TQ, ql = slot - (slot / a.TQ) * a.TQ;
        hp0[g] = pl * a.sh * a.WW + ql * a.sw;
    }

    floatx4 acc[NJ][NT];
#pragma unroll
    for (int g = 0; g < NJ; ++g)
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[g][t] = floatx4{0.f, 0.f, 0.f, 0.f};

    const int kstep_frags = a.ksteps * NT * 64;  // uint4 per chunk
    const uint4* wsrc = wpk + (int64_t)kb * a.nchunks * kstep_frags;
    uint4* wl = reinterpret_cast<uint4*>(lds + a.w_off);
    const int64_t HWi = (int64_t)a.H * a.W;
    const float* ximg = x + (int64_t)n * a.C * HWi;
    const int o = lane >> 4;

    for (int chunk = 0; chunk < a.nchunks; ++chunk) {
        const int c0 = chunk * CC;
        // ---- stage the x halo tile: one (pixel, channel octet) per item, lanes along W
        const int items = hw_halo * OCT;
        for (int it = tid; it < items; it += kThreads) {
            const int oc = it / hw_halo;
            const int hp = it - oc * hw_halo;
            const int hh = hp / a.WW, ww = hp - (hp / a.WW) * a.WW;
            const int h = h0 + hh, w = w0 + ww;
            const bool v = (h >= 0) && (h < a.H) && (w >= 0) && (w < a.W);
            const int cb = c0 + oc * 8;
            const float* src = ximg + (v ? ((int64_t)cb * HWi + (int64_t)h * a.W + w) : 0);
            uint32_t b[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) b[j] = (v && cb + j < a.C) ? __float_as_uint(src[j * HWi]) : 0u;
            uint4 hi, mid, lo;
            split3(b, hi, mid, lo);
            const int ad = x_addr<CC>(hp, oc);
            *reinterpret_cast<uint4*>(lds + ad) = hi;
            *reinterpret_cast<uint4*>(lds + a.plane + ad) = mid;
            *reinterpret_cast<uint4*>(lds + 2 * a.plane + ad) = lo;
        }
        // ---- stage this chunk's weight fragments
        const uint4* wc = wsrc + (int64_t)chunk * kstep_frags;
        for (int e = tid; e < kstep_frags; e += kThreads) wl[e] = wc[e];
        __syncthreads();

        for (int ks = 0; ks < a.ksteps; ++ks) {
            const int oi = ks * 4 + o;
            const int t = oi / OCT, coct = oi % OCT;
            const bool pad = t >= a.taps;
            const int toff = pad ? 0 : tapt[t];
            bf16x8 bw[NT];
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
                bw[nt] = __builtin_bit_cast(bf16x8, wl[(ks * NT + nt) * 64 + lane]);
#pragma unroll
            for (int g = 0; g < NJ; ++g) {
                const int ad = pad ? zero_off : x_addr<CC>(hp0[g] + toff, coct);
                const bf16x8 a0 = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(lds + ad));
                const bf16x8 a1 = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(lds + a.plane + ad));
                const bf16x8 a2 = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(lds + 2 * a.plane + ad));
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) {
                    acc[g][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bw[nt], acc[g][nt], 0, 0, 0);
                    acc[g][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bw[nt], acc[g][nt], 0, 0, 0);
                    acc[g][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2, bw[nt], acc[g][nt], 0, 0, 0);
                }
            }
        }
        __syncthreads();
    }

    // ---- epilogue: D[row = pixel 4*(lane>>4)+i][col = channel lane&15]
    const float scale = *scale_p;
    const int64_t PQ = (int64_t)a.P * a.Q;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        const int k = kb * 16 * NT + nt * 16 + (lane & 15);
        if (k >= a.K) continue;
        const float bk = bias ? bias[k] : 0.0f;
        float* yk = y + ((int64_t)n * a.K + k) * PQ;
#pragma unroll
        for (int g = 0; g < NJ; ++g) {
            const int i0 = (wave * NJ + g) * 16 + 4 * (lane >> 4);
            if (a.vec) {
                if (i0 >= npix) continue;
                const int pl = i0 / a.TQ, ql = i0 - (i0 / a.TQ) * a.TQ;
                const int pp = p0 + pl, qq = q0 + ql;
                if (pp >= a.P || qq >= a.Q) continue;
                float4 v;
                v.x = acc[g][nt][0] * scale + bk;
                v.y = acc[g][nt][1] * scale + bk;
                v.z = acc[g][nt][2] * scale + bk;
                v.w = acc[g][nt][3] * scale + bk;
                *reinterpret_cast<float4*>(yk + (int64_t)pp * a.Q + qq) = v;
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int idx = i0 + i;
                    if (idx >= npix) continue;
                    const int pl = idx / a.TQ, ql = idx - (idx / a.TQ) * a.TQ;
                    const int pp = p0 + pl, qq = q0 + ql;
                    if (pp >= a.P || qq >= a.Q) continue;
                    yk[(int64_t)pp * a.Q + qq] = acc[g][nt][i] * scale + bk;
                }
            }
        }
    }
}

// ------------------------------------------------------------------ planning --
static int cdiv(int a, int b) { return (a + b - 1) / b; }

static size_t x3_lds(const ConvPlan& p, int NT, int HH, int WW) {
    const int plane = HH * WW * p.SB + 16;
    return (size_t)3 * plane + (size_t)p.steps * NT * 1024 + 64 * sizeof(int);
}

bool plan_bf16x3(ConvPlan& p, int mode, int bits, int fsr) {
    if (mode == 0 || p.groups != 1) return false;
    if (bits < 1 || bits > 16) return false;
    const long lo = (long)fsr - (1L << (bits - 1)), hi = (long)fsr - 1;
    if (lo < -126 || hi > 127) return false;  // +-2^e must be a normal bf16
    p.taps = p.R * p.S;
    if (p.taps > 64) return false;
    p.CC = (p.taps == 1 && p.C > 16) ? 32 : 16;
    const int OCT = p.CC / 8;
    p.steps = cdiv(p.taps * OCT, 4);
    p.SB = 2 * p.CC;
    p.NT = p.K <= 16 ? 1 : (p.K <= 32 ? 2 : 4);
    p.kblocks = cdiv(p.K, 16 * p.NT);
    p.nchunks = cdiv(p.C, p.CC);

    // tile search (override: PO2Q_X3_TILE="NJ,TP,TQ", a tuning knob)
    int bestNJ = 0, bestTP = 0, bestTQ = 0;
    double best = 1e300;
    const char* env = getenv("PO2Q_X3_TILE");
    if (env) {
        int nj = 0, tp = 0, tq = 0;
        if (sscanf(env, "%d,%d,%d", &nj, &tp, &tq) == 3 && tp * tq == 64 * nj &&
            (nj == 1 || nj == 2 || nj == 4 || nj == 7 || nj == 8)) {
            bestNJ = nj; bestTP = tp; bestTQ = tq; best = 0;
        }
    }
    const int njs[] = {1, 2, 4, 7, 8};
    for (int nj : njs) {
        if (best == 0) break;
        if (nj * p.NT > 16) continue;
        const int px = 64 * nj;
        for (int tq = 1; tq <= std::min(p.Q, px); ++tq) {
            if (px % tq) continue;
            const int tp = px / tq;
            const int HH = (tp - 1) * p.sh + (p.R - 1) * p.dh + 1;
            const int WW = (tq - 1) * p.sw + (p.S - 1) * p.dw + 1;
            const size_t lds = x3_lds(p, p.NT, HH, WW);
            if (lds > 64 * 1024) continue;
            const int tP = cdiv(p.P, tp), tQ = cdiv(p.Q, tq);
            const double launched = (double)tP * tQ * px;
            const double waste = launched / ((double)p.P * p.Q);
            const double halo = (double)tP * tQ * HH * WW / ((double)p.P * p.Q * p.sh * p.sw);
            const int bpc = std::min<int>(8, (int)((160 * 1024) / lds));
            const int waves = std::min(bpc * 4, 32);
            double cost = waste + 0.35 * (halo - 1.0);
            if (waves < 8) cost += 0.15 * (8 - waves) / 4.0;
            if (tq % 16 && tq != p.Q) cost += 0.05;
            if (tq % 4) cost += 0.1;
            cost += 0.02 * (8.0 / nj);  // per-block fixed costs (barriers, weight staging)
            const double blocks = (double)p.N * p.kblocks * tP * tQ;
            if (blocks < 1024) cost += 0.5 * (1024 - blocks) / 1024;
            if (cost < best) {
                best = cost; bestNJ = nj; bestTP = tp; bestTQ = tq;
            }
        }
    }
    if (!bestNJ) return false;
    p.kind = KIND_BF16X3;
    p.NJ = bestNJ; p.TP = bestTP; p.TQ = bestTQ;
    p.tilesP = cdiv(p.P, p.TP);
    p.tilesQ = cdiv(p.Q, p.TQ);
    p.HH = (p.TP - 1) * p.sh + (p.R - 1) * p.dh + 1;
    p.WW = (p.TQ - 1) * p.sw + (p.S - 1) * p.dw + 1;
    p.plane = p.HH * p.WW * p.SB + 16;
    p.lds_bytes = x3_lds(p, p.NT, p.HH, p.WW);
    p.WWp = p.WW; p.PS = 0; p.MI = 0;
    // packed bf16 fragments: [kb][chunk][ks][nt][lane][8] -> 4-byte words
    p.packed_floats = (int64_t)p.kblocks * p.nchunks * p.steps * p.NT * 64 * 4;
    p.blocks = (int64_t)p.N * p.kblocks * p.tilesP * p.tilesQ;
    if (p.blocks > INT_MAX) return false;
    return true;
}

template <int CC, int NT, int NJ>
static hipError_t launch_x3(const ConvPlan& p, const X3Args& a, const float* x, const uint16_t* packed,
                            const float* scale, const float* bias, float* y, hipStream_t s) {
    hipLaunchKernelGGL((conv_bf16x3<CC, NT, NJ>), dim3((unsigned)p.blocks), dim3(kThreads), p.lds_bytes, s, x,
                       reinterpret_cast<const uint4*>(packed), scale, bias, y, a);
    return hipGetLastError();
}

template <int CC, int NT>
static hipError_t launch_x3_nj(const ConvPlan& p, const X3Args& a, const float* x, const uint16_t* packed,
                               const float* scale, const float* bias, float* y, hipStream_t s) {
    switch (p.NJ) {
        case 1: return launch_x3<CC, NT, 1>(p, a, x, packed, scale, bias, y, s);
        case 2: return launch_x3<CC, NT, 2>(p, a, x, packed, scale, bias, y, s);
        case 4: return launch_x3<CC, NT, 4>(p, a, x, packed, scale, bias, y, s);
        case 7: return launch_x3<CC, NT, 7>(p, a, x, packed, scale, bias, y, s);
        default: return launch_x3<CC, NT, 8>(p, a, x, packed, scale, bias, y, s);
    }
}

template <int CC>
static hipError_t launch_x3_nt(const ConvPlan& p, const X3Args& a, const float* x, const uint16_t* packed,
                               const float* scale, const float* bias, float* y, hipStream_t s) {
    switch (p.NT) {
        case 1: return launch_x3_nj<CC, 1>(p, a, x, packed, scale, bias, y, s);
        case 2: return launch_x3_nj<CC, 2>(p, a, x, packed, scale, bias, y, s);
        default: return launch_x3_nj<CC, 4>(p, a, x, packed, scale, bias, y, s);
    }
}

hipError_t launch_conv_bf16x3(const ConvPlan& p, const float* x, const uint16_t* packed, const float* scale,
                              const float* bias, float* y, hipStream_t s) {
    X3Args a;
    a.N = p.N; a.C = p.C; a.H = p.H; a.W = p.W; a.K = p.K; a.P = p.P; a.Q = p.Q;
    a.sh = p.sh; a.sw = p.sw; a.ph = p.ph; a.pw = p.pw; a.dh = p.dh; a.dw = p.dw; a.R = p.R; a.S = p.S;
    a.TP = p.TP; a.TQ = p.TQ; a.tilesP = p.tilesP; a.tilesQ = p.tilesQ; a.kblocks = p.kblocks;
    a.nchunks = p.nchunks; a.HH = p.HH; a.WW = p.WW; a.ksteps = p.steps; a.taps = p.taps;
    a.plane = p.plane;
    a.w_off = 3 * p.plane;
    a.tap_off = a.w_off + p.steps * p.NT * 1024;
    a.vec = (p.Q % 4 == 0 && p.TQ % 4 == 0) ? 1 : 0;
    a.nblocks = (int)p.blocks;
    a.remap = (p.blocks % 8 == 0) ? 1 : 0;
    if (p.CC == 16) return launch_x3_nt<16>(p, a, x, packed, scale, bias, y, s);
    return launch_x3_nt<32>(p, a, x, packed, scale, bias, y, s);
}

}  // namespace po2q
