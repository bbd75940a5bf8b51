// bf16x3 3x3 / stride-1 / pad-1 conv for SMALL images (CIFAR sizes: ResNet56 @32 runs its 52
// stride-1 convs at 32x32 x 16, 16x16 x 32 and 8x8 x 64), where a layer is a few MB and the row
// kernels' HBM streaming has nothing to stream: at 8x8 a 32-column strip is 3/4 empty and a
// layer is bound by the latency of its dependent load -> split -> MFMA -> store chain.
//
// Same arithmetic as every bf16x3 kernel (exact +-2^e bf16 weights x exact 3-way bf16 split
// of the fp32 activations, fp32 accumulation on v_mfma_f32_16x16x32_bf16; reference
// QuantizedConv2d.forward, models/quantized_conv.py:32-38), organised for latency:
//
//   * a block owns (image, segment of RB output rows, KG-th of the output channels); it loads
//     the segment's RB + 2 input rows (all C channels, zero-padded halo) with ONE batch of
//     independent loads per thread (8 channels of one pixel each), splits them and writes the
//     hi / mid / lo planes [(RB + 2) x (W + 2) padded pixels][C] bf16 to LDS -- one global
//     latency, one barrier, then no more global reads;
//   * each wave owns one 16-channel output tile (its B fragments: 3 tap rows x KS k-steps,
//     VGPR-resident, the row-kernel pack layout [r][ks][nt][lane][8] of pack_bf16x3_kernel) and
//     a share of the segment's 16-pixel groups (pixels flattened row-major, so a group may span
//     image rows: the A-fragment address of each lane is computed, not streamed);
//   * per group: 3 x KS k-steps, each 3 ds_read_b128 (hi, mid, lo) and 3 MFMAs; the eval BN
//     affine, residual and activation run in the store (each lane: 4 consecutive pixels of one
//     output channel, one float4).
// Plane layout [pixel][C] bf16 with the channel octets XOR-swizzled by the pixel index so that
// every LDS cycle of a fragment read is conflict-free for ANY starting pixel: ds_read_b128 serves
// the lane groups {0-3,12-15,20-27}, {4-11,16-19,28-31}, ... (MI355X_MICROARCH.md LDS table),
// i.e. pixels p..p+3 / p+12..p+15 of one octet with p+4..p+11 of the next.  C = 16 needs no
// swizzle, C = 32 flips octet bit 1 with pixel bit 2, C = 64 XORs 2 * (pixel >> 1 & 3)
// (exhaustive over every offset; the 8-byte-chunk and pixel>>k & mask swizzles were 2-way).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdint>

#include "../../include/po2q.h"
#include "po2q_epi.h"
#include "po2q_internal.h"
#include "po2q_x3_dev.h"

namespace po2q {

namespace {
constexpr int kImgThreads = 256;
constexpr int kImgItems = 4;                 // split items (pixel x channel octet) per thread and batch
constexpr size_t kImgLdsMax = 80 * 1024;     // 2 blocks per CU

template <int C>
__device__ __forceinline__ int img_addr(int pp, int oc) {
    if constexpr (C == 16)
        return pp * 32 + 16 * oc;
    else if constexpr (C == 32)
        return pp * 64 + 16 * (oc ^ (((pp >> 2) & 1) << 1));
    else
        return pp * 128 + 16 * (oc ^ (((pp >> 1) & 3) << 1));
}
}  // namespace

struct ImgArgs {
    int N, H, W, K;
    int RB, nseg, KG;  // output rows per block, row segments per image, output-channel groups
    int PW, PL, ZO;    // padded row pitch (W + 2), bytes per plane, zero slot offset in a plane
    int NT;            // 16-channel output tiles of K (packed layout)
    const float* ps;   // eval BN affine (NULL: none)
    const float* pb;
    const float* res;  // residual [N, K, H, W] (NULL: none)
    int act;
};

// C: input channels (16, 32, 64); NTB: output tiles per block (waves per tile: 4 / NTB)
template <int C, int NTB, bool EPI>
__global__ __launch_bounds__(kImgThreads, 2) void conv_img(const float* __restrict__ x, const uint4* __restrict__ wpk,
                                                           const float* __restrict__ scale_p,
                                                           const float* __restrict__ bias, float* __restrict__ y,
                                                           ImgArgs a) {
    constexpr int KS = C == 16 ? 2 : 3 * (C / 32);  // k-steps per tap row (row-kernel pack layout)
    constexpr int NO = C / 8;                       // channel octets per pixel
    constexpr int WPT = 4 / NTB;                    // waves sharing one output tile
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    int b = blockIdx.x;
    const int kg = b % a.KG;
    b /= a.KG;
    const int seg = b % a.nseg;
    const int n = b / a.nseg;
    const int r0 = seg * a.RB;
    const int rbe = min(a.RB, a.H - r0);
    const int nt = kg * NTB + wave % NTB;
    const int gsub = wave / NTB;

    // this wave's B fragments (L2-resident pack), in flight with the x loads below
    bf16x8 bw[3 * KS];
#pragma unroll
    for (int f = 0; f < 3 * KS; ++f) bw[f] = __builtin_bit_cast(bf16x8, wpk[(int64_t)(f * a.NT + nt) * 64 + lane]);

    // ---- load + split: item = (channel octet, padded row, padded column), column fastest so
    // consecutive lanes read consecutive pixels of each channel
    const int rows = rbe + 2;
    const int nitems = rows * a.PW * NO;
    const int HWs = a.H * a.W;
    const float* xn = x + (int64_t)n * C * HWs;
    for (int base = 0; base < nitems; base += kImgThreads * kImgItems) {
        uint32_t v[kImgItems][8];
        int dst[kImgItems];
#pragma unroll
        for (int i = 0; i < kImgItems; ++i) {
            const int it = base + i * kImgThreads + tid;
            const bool ok = it < nitems;
            const int pc = it % a.PW, t = it / a.PW;
            const int rr = t % rows, oc = t / rows;
            const int h = r0 - 1 + rr, xc = pc - 1;
            const bool inb = ok && h >= 0 && h < a.H && xc >= 0 && xc < a.W;
            const float* src = xn + (int64_t)(8 * oc) * HWs + (inb ? h * a.W + xc : 0);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[i][e] = inb ? __float_as_uint(src[(int64_t)e * HWs]) : 0u;
            dst[i] = ok ? img_addr<C>(rr * a.PW + pc, oc) : -1;
        }
#pragma unroll
        for (int i = 0; i < kImgItems; ++i) {
            if (dst[i] < 0) continue;
            uint4 hi, mid, lo;
            split3(v[i], hi, mid, lo);
            *reinterpret_cast<uint4*>(lds + dst[i]) = hi;
            *reinterpret_cast<uint4*>(lds + a.PL + dst[i]) = mid;
            *reinterpret_cast<uint4*>(lds + 2 * a.PL + dst[i]) = lo;
        }
    }
    if (tid < 3) *reinterpret_cast<uint4*>(lds + tid * a.PL + a.ZO) = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();

    // ---- MFMAs: lane -> pixel p of the group (A row), k-octet group g4
    const float scale = *scale_p;
    const int p = lane & 15, g4 = lane >> 4;
    const int npx = rbe * a.W;
    const int ngroups = (npx + 15) >> 4;
    const int k = 16 * nt + (lane & 15);
    const float bk = bias ? bias[k] : 0.0f;
    const float eps_ = (EPI && a.ps) ? a.ps[k] : 1.0f;
    const float epb_ = (EPI && a.pb) ? a.pb[k] : 0.0f;
    for (int grp = gsub; grp < ngroups; grp += WPT) {
        const int f = 16 * grp + p;
        const int fo = f < npx ? f : 0;  // past the segment: a valid pixel, the result is not stored
        const int oy = fo / a.W, ox = fo - oy * a.W;
        const int pp0 = oy * a.PW + ox;  // padded pixel of tap (0, 0)
        floatx4 acc = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int r = 0; r < 3; ++r) {
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                int ad;
                if constexpr (C == 16) {
                    // ks 0: taps (s0 | s1), ks 1: (s2 | zero) -- the row-kernel layout
                    const int s = ks == 0 ? (g4 >> 1) : 2;
                    ad = (ks == 1 && g4 >= 2) ? a.ZO : img_addr<C>(pp0 + r * a.PW + s, g4 & 1);
                } else {
                    const int s = ks % 3;
                    ad = img_addr<C>(pp0 + r * a.PW + s, (ks / 3) * 4 + g4);
                }
                const bf16x8 ah = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(lds + ad));
                const bf16x8 am = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(lds + a.PL + ad));
                const bf16x8 al = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(lds + 2 * a.PL + ad));
                const bf16x8 bb = bw[r * KS + ks];
                acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bb, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bb, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bb, acc, 0, 0, 0);
            }
        }
        // D[pixel 4 g4 + e][channel lane & 15]: 4 consecutive pixels of one row (W % 4 == 0)
        const int f0 = 16 * grp + 4 * g4;
        if (f0 >= npx) continue;
        const int sy = f0 / a.W, sx = f0 - sy * a.W;
        const int64_t off = (((int64_t)n * a.K + k) * a.H + r0 + sy) * a.W + sx;
        float vv[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            float u = acc[e] * scale + bk;
            if constexpr (EPI) u = u * eps_ + epb_;
            vv[e] = u;
        }
        if constexpr (EPI) {
            if (a.res) {
                const float4 rv = *reinterpret_cast<const float4*>(a.res + off);
                vv[0] += rv.x; vv[1] += rv.y; vv[2] += rv.z; vv[3] += rv.w;
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) vv[e] = epi_act(vv[e], a.act);
        }
        *reinterpret_cast<float4*>(y + off) = make_float4(vv[0], vv[1], vv[2], vv[3]);
    }
}

// ------------------------------------------------------------------ planning --
static size_t img_plane(int C, int rb, int W) { return (size_t)(rb + 2) * (W + 2) * 2 * C + 16; }

static bool img_plan_one(ConvPlan& p, int rb, int kg) {
    const int NT = p.K / 16;
    p.kind = KIND_BF16X3_IMG;
    p.vrx = 0;
    p.CC = p.C == 16 ? 16 : 32;
    p.nchunks = p.C / p.CC;
    p.steps = p.C == 16 ? 2 : 3 * p.nchunks;  // k-steps per tap row
    p.NT = NT;
    p.NJ = 0;
    p.MI = 0;
    p.taps = 9;
    p.TP = rb;
    p.TQ = p.W;
    p.tilesP = (p.H + rb - 1) / rb;
    p.tilesQ = 1;
    p.kblocks = kg;
    p.HH = rb + 2;
    p.WW = p.WWp = p.W + 2;
    p.PS = 0;
    p.SB = 2 * p.C;
    p.plane = (int)img_plane(p.C, rb, p.W);
    p.pd = 0;
    p.nts = 0;
    p.fp = 0;
    p.dma_d0 = p.dma_nck = p.dma_ni = p.dma_nw = p.dma_waves = p.dma_ov = 0;
    p.packed_floats = (int64_t)3 * p.steps * NT * 64 * 4;
    p.lds_bytes = 3 * (size_t)p.plane;
    p.blocks = (int64_t)p.N * p.tilesP * kg;
    return p.lds_bytes <= kImgLdsMax && p.blocks <= INT_MAX;
}

void img_candidates(const ConvPlan& b, int mode, int bits, int fsr, std::vector<PlanCand>& out) {
    out.clear();
    if (mode == 0 || b.groups != 1) return;
    if (bits < 1 || bits > 16) return;
    const long lo = (long)fsr - (1L << (bits - 1)), hi = (long)fsr - 1;
    if (lo < -126 || hi > 127) return;  // +-2^e must be a normal bf16
    if (b.R != 3 || b.S != 3 || b.sh != 1 || b.sw != 1 || b.ph != 1 || b.pw != 1 || b.dh != 1 || b.dw != 1) return;
    if (!(b.C == 16 || b.C == 32 || b.C == 64) || !(b.K == 16 || b.K == 32 || b.K == 64)) return;
    if (b.W % 4 != 0 || b.W > 64 || b.H < 1) return;
    if ((int64_t)b.N * b.C * b.H * b.W >= (1LL << 31) || (int64_t)b.N * b.K * b.H * b.W >= (1LL << 31)) return;
    const int NT = b.K / 16;
    int last_rb = -1;
    for (int div : {1, 2, 4, 8}) {
        const int rb = (b.H + div - 1) / div;
        if (rb == last_rb) continue;
        last_rb = rb;
        for (int kg : {1, 2, 4}) {
            if (NT % kg != 0) continue;
            ConvPlan p = b;
            if (!img_plan_one(p, rb, kg)) continue;
            // cost: rounds of co-resident blocks (2 per CU) x a block's dependent chain (one
            // load latency, the split, the busiest wave's MFMAs), in ~cycles
            const int KS = p.steps;
            const int64_t groups = ((int64_t)rb * b.W + 15) / 16;
            const int wpt = 4 / (NT / kg);
            const double mfma = (double)((groups + wpt - 1) / wpt) * 9.0 * KS * 16.0;
            const double split = (double)(rb + 2) * (b.W + 2) * (b.C / 8) / kImgThreads * 60.0;
            const double chain = 2500.0 + split + mfma;
            const double rounds = std::ceil((double)p.blocks / 512.0);
            PlanCand c;
            c.plan = p;
            c.cost = rounds * chain;
            out.push_back(c);
        }
    }
    std::stable_sort(out.begin(), out.end(), [](const PlanCand& u, const PlanCand& v) { return u.cost < v.cost; });
}

template <int C, int NTB>
static hipError_t launch_img_t(const ConvPlan& p, const ImgArgs& a, const float* x, const uint4* wp,
                               const float* scale, const float* bias, float* y, bool epi, hipStream_t s) {
    const dim3 grid((unsigned)p.blocks), block(kImgThreads);
    if (epi)
        hipLaunchKernelGGL((conv_img<C, NTB, true>), grid, block, p.lds_bytes, s, x, wp, scale, bias, y, a);
    else
        hipLaunchKernelGGL((conv_img<C, NTB, false>), grid, block, p.lds_bytes, s, x, wp, scale, bias, y, a);
    return hipGetLastError();
}

hipError_t launch_conv_img(const ConvPlan& p, const float* x, const uint16_t* packed, const float* scale,
                           const float* bias, float* y, const float* ps, const float* pb, const float* res, int act,
                           hipStream_t s) {
    if (p.kind != KIND_BF16X3_IMG || p.lds_bytes > kImgLdsMax || p.K % 16 != 0 || p.W % 4 != 0 ||
        p.NT % p.kblocks != 0 || p.TP < 1 || p.tilesP != (p.H + p.TP - 1) / p.TP ||
        p.blocks != (int64_t)p.N * p.tilesP * p.kblocks || p.plane != (int)img_plane(p.C, p.TP, p.W))
        return hipErrorInvalidValue;
    ImgArgs a;
    a.N = p.N; a.H = p.H; a.W = p.W; a.K = p.K;
    a.RB = p.TP; a.nseg = p.tilesP; a.KG = p.kblocks;
    a.PW = p.W + 2;
    a.PL = p.plane;
    a.ZO = p.plane - 16;
    a.NT = p.NT;
    a.ps = ps; a.pb = pb; a.res = res; a.act = act;
    const bool epi = ps || pb || res || act != 0;
    const uint4* wp = reinterpret_cast<const uint4*>(packed);
    const int ntb = p.NT / p.kblocks;
#define PO2Q_IMG(c, t) \
    if (p.C == c && ntb == t) return launch_img_t<c, t>(p, a, x, wp, scale, bias, y, epi, s);
    PO2Q_IMG(16, 1) PO2Q_IMG(16, 2) PO2Q_IMG(16, 4)
    PO2Q_IMG(32, 1) PO2Q_IMG(32, 2) PO2Q_IMG(32, 4)
    PO2Q_IMG(64, 1) PO2Q_IMG(64, 2) PO2Q_IMG(64, 4)
#undef PO2Q_IMG
    return hipErrorInvalidValue;
}

}  // namespace po2q
