// bf16x3 row-streaming conv, output channels split across the waves of a block:
// 3x3 / stride 1 / pad 1, C = K = 64 (ResNet56 stage 3: 17 of its 56 qconvs) and
// C = K = 32 (stage 2: 17 more).
//
// Same arithmetic as the other bf16x3 kernels (exact +-2^e bf16 weights x exact
// 3-way bf16 split of the fp32 activations, fp32 accumulation on
// v_mfma_f32_16x16x32_bf16; reference: QuantizedConv2d.forward,
// models/quantized_conv.py:32-38).  Stage 3 is MFMA-heavy (576 MACs per output
// element), so the layout is chosen for the matrix cores:
//
//   * a 4-wave block owns (image, strip of 32 output columns, segment of rows) and
//     marches down it one halo row at a time, like po2q_conv_rows.hip.  C = 64: wave w
//     computes output channels 16w .. 16w+15 for both 16-column groups of the strip;
//     C = 32: wave w computes channels 16(w&1) .. +15 for column group w>>1;
//   * each wave's B fragments (3 tap rows x C/32 channel chunks x 3 taps bf16x8)
//     stay in VGPRs for the kernel's lifetime -- no weight traffic in the loop;
//   * per halo row, wave w LDS-DMAs channels [wC/4, (w+1)C/4) of the strip (C/32 x
//     1 KiB, 128-byte runs) plus C/2 of the 2C halo-column values into a 2-slot raw
//     ring, and splits exactly what it loaded into the shared hi / mid / lo planes
//     (double-buffered):
//     the DMA -> split dependency is wave-local (an exact vmcnt wait), and ONE block
//     barrier per row publishes the planes;
//   * every A fragment read from the planes feeds 3 MFMAs (the three output rows the
//     halo row touches); three accumulator slots rotate; loop unrolled by 6.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdlib>
#include <type_traits>
#include <vector>

#include "po2q_epi.h"
#include "po2q_internal.h"
#include "po2q_rows_dev.h"
#include "po2q_x3_dev.h"

namespace po2q {

namespace {

constexpr int kKSW = 32;                       // strip width (2 pixel groups of 16)
constexpr int kKWC = kKSW + 2;                 // halo columns
template <int C> constexpr int kKPlane = kKWC * C * 2;          // bytes per bf16 plane
template <int C> constexpr int kKRawInt = C * kKSW * 4;        // raw interior [C][32] fp32
template <int C> constexpr int kKRawSlot = kKRawInt<C> + 4 * 256;  // + 4 waves x 64 halo dwords
template <int C, int PD> constexpr int kKLds = 2 * 3 * kKPlane<C> + PD * kKRawSlot<C>;

// byte offset of (halo column hc, channel octet oct) in a plane, 2C bytes per pixel;
// octets XOR-swizzled by the column (C = 64: 8 octets, C = 32: the x_addr<32> layout)
// so consecutive pixels of one octet spread over the bank quads
template <int C>
__device__ __forceinline__ int k_addr(int hc, int oct) {
    if constexpr (C == 64)
        return hc * 128 + ((oct ^ (hc & 7)) << 4);
    else
        return x_addr<32>(hc, oct);
}

}  // namespace

struct RowsKArgs {
    int N, H, W, P, Q;
    int RB, nseg, nstrip, items;
    int remap;
    const float* ps;  // fused epilogue (EPI): y = act(y * ps[k] + pb[k]); either may be NULL
    const float* pb;
    int act;
};

// PD: halo rows in flight per wave (raw ring slots), 2 or 3
// DBG (diagnostic builds only, -DPO2Q_ROWS_DIAG): 1 = halo-column DMAs read nothing
// (out-of-range offsets; timing only, outputs wrong).  Product builds: DBG = 0.
template <int C, int PD, bool EPI = false, int DBG = 0>
__global__ __launch_bounds__(kThreads, C == 64 ? 3 : 4) void conv_rowsk(const float* __restrict__ x, const uint4* __restrict__ wpk,
                                                          const float* __restrict__ scale_p,
                                                          const float* __restrict__ bias, float* __restrict__ y,
                                                          RowsKArgs a) {
    constexpr int K = C;
    constexpr int NCH = C / 32;        // 32-channel chunks (k-steps per tap: one per chunk)
    constexpr int KSC = 3 * NCH;       // k-steps per tap row
    constexpr int WN = K / 16;         // waves along the output channels
    constexpr int NGW = 2 * WN / 4;    // 16-column groups per wave (2 for C = 64, 1 for C = 32)
    constexpr int DPW = C / 32;        // interior DMAs per wave per row (1 KiB each)
    constexpr int HPW = C / 2;         // halo values per wave per row
    constexpr int PL = kKPlane<C>;
    constexpr int RAWI = kKRawInt<C>;
    constexpr int RAWS = kKRawSlot<C>;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wn = wave % WN;                    // output-channel tile of this wave
    const int g0 = (wave / WN) * NGW;            // first column group of this wave
    unsigned char* planes = lds;                 // 2 buffers x 3 planes
    unsigned char* raw = lds + 2 * 3 * PL;       // PD slots

    int blk = blockIdx.x;
    if (a.remap) blk = (blk & 7) * (int)(gridDim.x >> 3) + (blk >> 3);
    const int item = blk;  // one item per block
    if (item >= a.items) return;
    const int strip = item % a.nstrip;
    const int t0 = item / a.nstrip;
    const int seg = t0 % a.nseg;
    const int n = t0 / a.nseg;
    const int q0 = strip * kKSW;
    const int p0 = seg * a.RB;
    const int rbe = min(a.RB, a.P - p0);
    const int nrows = rbe + 2;

    // ---- this wave's weights: B[r][ks = chunk*3 + s] for output channels 16w..16w+15
    bf16x8 bw[3][KSC];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int ks = 0; ks < KSC; ++ks)
            bw[r][ks] = __builtin_bit_cast(bf16x8, wpk[((r * KSC + ks) * WN + wn) * 64 + lane]);
    const int kout = 16 * wn + (lane & 15);
    float bk = bias ? bias[kout] : 0.0f;
    float eps_ = (EPI && a.ps) ? a.ps[kout] : 1.0f;
    float epb_ = (EPI && a.pb) ? a.pb[kout] : 0.0f;
    const float scale = *scale_p;
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int ks = 0; ks < KSC; ++ks) asm volatile("s_waitcnt vmcnt(0)" : "+v"(bw[r][ks]));
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(bk), "+v"(eps_), "+v"(epb_));
    auto outv = [&](float accv) __attribute__((always_inline)) {
        const float v = accv * scale + bk;
        if constexpr (EPI)
            return epi_act(v * eps_ + epb_, a.act);
        else
            return v;
    };

    // ---- DMA: wave w, instruction i: lane l -> channel (C/4)w + 8i + (l >> 3), columns
    // 4*(l & 7) .. +3, landing at raw[c][col] (row-major, 128 B per channel); halo:
    // lanes 0..C/2-1 of wave w -> value v = (C/2)w + lane: side v / C, channel v % C
    const int HW = a.H * a.W;
    const uint32_t cstride = (uint32_t)HW * 4u;
    const __amdgpu_buffer_rsrc_t rs = rows_rsrc(x + (int64_t)n * C * HW, C * HW * 4);
    const int cb = lane & 7;
    const int gq4 = q0 + 4 * cb;
    const bool qi_ok = gq4 < a.W;
    const uint32_t vi0 = (uint32_t)((C / 4) * wave + (lane >> 3)) * cstride + (uint32_t)gq4 * 4u;
    const uint32_t soff1 = 8u * cstride;
    const int hv = HPW * wave + lane;
    const int hside = hv / C, hch = hv % C;
    const int gqh = hside ? q0 + kKSW : q0 - 1;
    const bool qh_ok = lane < HPW && gqh >= 0 && gqh < a.W;
    const uint32_t vh0 = (uint32_t)hch * cstride + (uint32_t)gqh * 4u;
    const uint32_t raw_lds = (uint32_t)(uintptr_t)raw;

    // ---- split: lane -> (column sc, channel octet DPW*w + so), reading what this wave
    // loaded (C = 32: lanes 32..63 idle)
    const int sc = lane & 31, so = lane >> 5;
    const bool sl_ok = so < DPW;
    const int oct = DPW * wave + (sl_ok ? so : 0);
    const int rd0 = (8 * oct) * (kKSW * 4) + sc * 4;
    const int wa_i = k_addr<C>(sc + 1, oct);
    const int wa_h = k_addr<C>(hside ? kKWC - 1 : 0, hch >> 3) + (hch & 7) * 2;

    // ---- A fragment offsets: (group grp, chunk ch, tap s): pixel 16grp + p + s, octet 4ch + g
    int aoff[NGW][KSC];
    {
        const int p = lane & 15, g = lane >> 4;
#pragma unroll
        for (int grp = 0; grp < NGW; ++grp)
#pragma unroll
            for (int ch = 0; ch < NCH; ++ch)
#pragma unroll
                for (int s = 0; s < 3; ++s)
                    aoff[grp][ch * 3 + s] = k_addr<C>(16 * (g0 + grp) + p + s, 4 * ch + g);
    }

    auto load_row = [&](int sl, int j) __attribute__((always_inline)) {
        const int h = p0 - 1 + j;
        const bool hok = j < nrows && h >= 0 && h < a.H;
        const uint32_t roff = (uint32_t)(hok ? h : 0) * (uint32_t)a.W * 4u;
        const uint32_t vo = (hok && qi_ok) ? vi0 + roff : 0x7fffffffu;
        const uint32_t base = raw_lds + (uint32_t)(sl * RAWS);
#pragma unroll
        for (int i = 0; i < DPW; ++i) rows_dma16(rs, vo, i * soff1, base + (uint32_t)(DPW * wave + i) * 1024u);
        const uint32_t voh = (hok && qh_ok && !(DBG & 1)) ? vh0 + roff : 0x7fffffffu;
        rows_dma4(rs, voh, base + (uint32_t)RAWI + (uint32_t)wave * 256u);
    };
    // vm ops issued after a row's DMAs (step j-PD) until row j is split: that step's
    // stores, then per later step the DMAs of one more row and that step's stores
    constexpr int VMW = (PD - 1) * (DPW + 1 + NGW) + NGW;
    const int PQ = a.P * a.Q;
    const __amdgpu_buffer_rsrc_t ry = rows_rsrc(y + (int64_t)n * K * PQ, K * PQ * 4);

    floatx4 acc[3][NGW];
#pragma unroll
    for (int sl = 0; sl < 3; ++sl)
#pragma unroll
        for (int grp = 0; grp < NGW; ++grp) acc[sl][grp] = floatx4{0.f, 0.f, 0.f, 0.f};

    auto step = [&](auto S_, int j) __attribute__((always_inline)) {
        constexpr int S6 = decltype(S_)::value;
        constexpr int S = S6 % 3;   // accumulator rotation
        constexpr int B2 = S6 % 2;  // plane buffer
        constexpr int RS = S6 % PD; // raw slot
        unsigned char* pb = planes + B2 * 3 * PL;
        const unsigned char* rw = raw + RS * RAWS;
        rows_wait<VMW>();  // this wave's DMAs of row j have landed
        {
            uint32_t b8[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) b8[e] = *reinterpret_cast<const uint32_t*>(rw + rd0 + e * (kKSW * 4));
            uint4 hi, mid, lo;
            split3(b8, hi, mid, lo);
            if (sl_ok) {
                *reinterpret_cast<uint4*>(pb + wa_i) = hi;
                *reinterpret_cast<uint4*>(pb + PL + wa_i) = mid;
                *reinterpret_cast<uint4*>(pb + 2 * PL + wa_i) = lo;
            }
            if (lane < HPW) {
                uint16_t h16, m16, l16;
                split1(*reinterpret_cast<const uint32_t*>(rw + RAWI + wave * 256 + 4 * lane), h16, m16, l16);
                *reinterpret_cast<uint16_t*>(pb + wa_h) = h16;
                *reinterpret_cast<uint16_t*>(pb + PL + wa_h) = m16;
                *reinterpret_cast<uint16_t*>(pb + 2 * PL + wa_h) = l16;
            }
        }
        // publish the planes: LDS writes done, then the block barrier (no memory fence:
        // the prefetches and stores in flight must not be waited for)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        // refill the raw slot this wave just split (its own data only)
        load_row(RS, j + PD);
        // MFMAs: halo row j feeds output halo-index j+1 (r=0), j (r=1), j-1 (r=2)
        constexpr int SL[3] = {(S + 1) % 3, S, (S + 2) % 3};
#pragma unroll
        for (int ks = 0; ks < KSC; ++ks) {
            bf16x8 af[3][NGW];
#pragma unroll
            for (int pl = 0; pl < 3; ++pl)
#pragma unroll
                for (int grp = 0; grp < NGW; ++grp)
                    af[pl][grp] = __builtin_bit_cast(
                        bf16x8, *reinterpret_cast<const uint4*>(pb + pl * PL + aoff[grp][ks]));
#pragma unroll
            for (int rr = 0; rr < 3; ++rr)
#pragma unroll
                for (int pl = 0; pl < 3; ++pl)
#pragma unroll
                    for (int grp = 0; grp < NGW; ++grp)
                        acc[SL[rr]][grp] =
                            __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[pl][grp], bw[rr][ks], acc[SL[rr]][grp], 0, 0, 0);
        }
        // output halo-index j-1 (row p0 + j - 2) is complete
        constexpr int D = (S + 2) % 3;
        const int o = p0 + j - 2;
        const bool orow = j >= 2 && o < p0 + rbe;
        const uint32_t yk = (uint32_t)kout * (uint32_t)PQ + (uint32_t)(orow ? o : 0) * a.Q;
#pragma unroll
        for (int grp = 0; grp < NGW; ++grp) {
            const int q = q0 + 16 * (g0 + grp) + 4 * (lane >> 4);
            floatx4 v;
            v[0] = outv(acc[D][grp][0]);
            v[1] = outv(acc[D][grp][1]);
            v[2] = outv(acc[D][grp][2]);
            v[3] = outv(acc[D][grp][3]);
            rows_store(ry, (orow && q < a.Q) ? (yk + (uint32_t)q) * 4u : 0x7fffffffu, v);
            acc[D][grp] = floatx4{0.f, 0.f, 0.f, 0.f};
        }
    };

    {
        const floatx4 z = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int r = 0; r < PD; ++r) {
            load_row(r, r);
#pragma unroll
            for (int i = 0; i < NGW; ++i) rows_store(ry, 0x7fffffffu, z);
        }
    }
    for (int j = 0; j < nrows; j += 6) {
        step(std::integral_constant<int, 0>{}, j);
        step(std::integral_constant<int, 1>{}, j + 1);
        step(std::integral_constant<int, 2>{}, j + 2);
        if (j + 3 >= nrows) break;
        step(std::integral_constant<int, 3>{}, j + 3);
        step(std::integral_constant<int, 4>{}, j + 4);
        step(std::integral_constant<int, 5>{}, j + 5);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // trailing DMAs land before the wave ends
}

// ------------------------------------------------------------------ planning --
// Candidates for 3x3 / s1 / p1 / C = K = 64 (plan kind bf16x3_rows with vrx = 1:
// output channels across the block's waves).  Weight pack: the row layout
// [r][ks = chunk*3 + s][nt][lane][8] (po2q_quant.hip, CC = 32, 2 chunks).
void rowsk_candidates(const ConvPlan& b, int mode, int bits, int fsr, std::vector<PlanCand>& out) {
    if (mode == 0 || b.groups != 1) return;
    if (bits < 1 || bits > 16) return;
    const long lo = (long)fsr - (1L << (bits - 1)), hi = (long)fsr - 1;
    if (lo < -126 || hi > 127) return;
    if (b.R != 3 || b.S != 3 || b.sh != 1 || b.sw != 1 || b.ph != 1 || b.pw != 1 || b.dh != 1 || b.dw != 1) return;
    if (!((b.C == 64 && b.K == 64) || (b.C == 32 && b.K == 32)) || b.Q % 4 != 0) return;
    if ((int64_t)b.C * b.H * b.W * 4 >= (1LL << 31) || (int64_t)b.K * b.P * b.Q * 4 >= (1LL << 31)) return;
    ConvPlan p = b;
    p.kind = KIND_BF16X3_ROWS;
    p.vrx = 1;
    p.CC = 32;
    p.nchunks = b.C / 32;
    p.NT = b.K / 16;
    p.NJ = 2;
    p.TQ = kKSW;
    p.steps = 3 * p.nchunks;  // k-steps per tap row (chunks x 3 taps)
    p.kblocks = 1;
    p.taps = 9;
    p.PS = 0; p.MI = 0; p.pd = 2;
    p.dma_d0 = p.dma_nck = p.dma_ni = p.dma_nw = p.dma_waves = p.dma_ov = 0;
    p.HH = 0; p.WW = p.WWp = kKWC;
    p.SB = 2 * b.C;
    p.plane = b.C == 64 ? kKPlane<64> : kKPlane<32>;
    p.packed_floats = (int64_t)3 * p.steps * p.NT * 64 * 4;
    p.tilesQ = (p.Q + kKSW - 1) / kKSW;
    // blocks resident per chip: 3 per CU for C = 64 (VGPR budget), 4 for C = 32
    const int slots = 256 * (b.C == 64 ? 3 : 4);
    std::vector<std::pair<double, int>> rbs;
    for (int rb = 4; rb <= p.P; ++rb) {
        const int nseg = (p.P + rb - 1) / rb;
        if (rb != (p.P + nseg - 1) / nseg) continue;
        const int64_t items = (int64_t)p.N * nseg * p.tilesQ;
        if (items > INT_MAX / 2) continue;
        rbs.push_back({(double)((items + slots - 1) / slots) * (rb + 2), rb});
    }
    std::sort(rbs.begin(), rbs.end());
    for (int pd : {3, 2})  // prefetch depth (halo rows in flight); 3 slots fit 3 blocks / CU
        for (int i = 0; i < (int)rbs.size() && i < 3; ++i) {
            ConvPlan c = p;
            c.pd = pd;
            c.lds_bytes = b.C == 64 ? (pd == 3 ? kKLds<64, 3> : kKLds<64, 2>) : (pd == 3 ? kKLds<32, 3> : kKLds<32, 2>);
            c.TP = rbs[i].second;
            c.tilesP = (p.P + c.TP - 1) / c.TP;
            const int64_t items = (int64_t)p.N * c.tilesP * c.tilesQ;
            c.blocks = (items + 7) / 8 * 8;
            out.push_back({0.9 + 0.001 * i + (pd == 2 ? 0.01 : 0.0), c});
        }
}

hipError_t launch_conv_rowsk(const ConvPlan& p, const float* x, const uint16_t* packed, const float* scale,
                             const float* bias, float* y, hipStream_t s, const float* ps, const float* pb,
                             int act, bool epi) {
    RowsKArgs a;
    a.N = p.N; a.H = p.H; a.W = p.W; a.P = p.P; a.Q = p.Q;
    a.RB = p.TP; a.nseg = p.tilesP; a.nstrip = p.tilesQ;
    a.items = p.N * p.tilesP * p.tilesQ;
    a.remap = (p.blocks % 8 == 0) ? 1 : 0;
    a.ps = ps;
    a.pb = pb;
    a.act = act;
#define PO2Q_RK(c, d, e)                                                                                    \
    if (p.C == c && p.pd == d && epi == e) {                                                                 \
        hipLaunchKernelGGL((conv_rowsk<c, d, e>), dim3((unsigned)p.blocks), dim3(kThreads), p.lds_bytes, s, x, \
                           reinterpret_cast<const uint4*>(packed), scale, bias, y, a);                        \
        return hipGetLastError();                                                                            \
    }
#ifdef PO2Q_ROWS_DIAG
    if (getenv("PO2Q_ROWSK_DEBUG") && atoi(getenv("PO2Q_ROWSK_DEBUG")) == 1) {
        if (p.C == 64 && p.pd == 3) {
            hipLaunchKernelGGL((conv_rowsk<64, 3, false, 1>), dim3((unsigned)p.blocks), dim3(kThreads), p.lds_bytes,
                               s, x, reinterpret_cast<const uint4*>(packed), scale, bias, y, a);
            return hipGetLastError();
        }
        if (p.C == 32 && p.pd == 2) {
            hipLaunchKernelGGL((conv_rowsk<32, 2, false, 1>), dim3((unsigned)p.blocks), dim3(kThreads), p.lds_bytes,
                               s, x, reinterpret_cast<const uint4*>(packed), scale, bias, y, a);
            return hipGetLastError();
        }
    }
#endif
    PO2Q_RK(64, 3, false) PO2Q_RK(64, 2, false) PO2Q_RK(32, 3, false) PO2Q_RK(32, 2, false)
    PO2Q_RK(64, 3, true) PO2Q_RK(64, 2, true) PO2Q_RK(32, 3, true) PO2Q_RK(32, 2, true)

#undef PO2Q_RK
    return hipErrorInvalidValue;
}

}  // namespace po2q
