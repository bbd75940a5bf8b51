// bf16x3 full-row-block conv for 3x3 / stride 1 / pad 1 with C = K = 16 (ResNet56 stage 1:
// 18 of its 56 quantized convs, the dominant layer of the bench).
//
// Same arithmetic as the other bf16x3 kernels (exact +-2^e bf16 weights x exact 3-way bf16
// split of the fp32 activations, fp32 accumulation on v_mfma_f32_16x16x32_bf16; reference:
// QuantizedConv2d.forward, models/quantized_conv.py:32-38) and the same per-wave compute as
// po2q_conv_rows.hip (a wave owns 32 output columns, row reuse over the 3 tap rows, 3
// rotating accumulator slots, transposed 128-byte-run stores).  What changes is the walk:
//
//   * one BLOCK owns (image, segment of RB output rows) across the WHOLE width: wave w of
//     the W/32 waves owns columns 32w .. 32w+31;
//   * per halo row the block LDS-DMAs the row's 16 channel runs (16 x W fp32, one 4W-byte
//     run per channel) into a raw ring slot [16][Wp]; each wave issues 2 of the Wp/16
//     1-KiB instructions, so the memory system sees whole-row runs, not 128-byte strips;
//   * no halo-column DMA: a wave reads its two halo columns straight from the neighbours'
//     part of the shared raw row (r02 probe: the per-strip halo dword DMA cost ~5 % of the
//     layer; tools/copy_probe.hip mode 2);
//   * one s_barrier per row: each wave waits for its own DMAs (exact vmcnt), the barrier
//     makes the whole row visible, and the slot of the previous row (split by every wave
//     before this barrier) is refilled right after it -- PD - 1 rows stay in flight.
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
constexpr int kFSW = 32;                 // output columns per wave
constexpr int kFWC = kFSW + 2;           // halo columns per wave
constexpr int kFPlane = kFWC * 16 * 2 + 32;  // bytes per bf16 plane (+ zero slot, pad)
constexpr int kFWBytes = 3 * 2 * 1024;   // B fragments: 3 tap rows x 2 k-steps (C = 16, NT = 1)
}  // namespace

struct RowsFArgs {
    int N, H, W, P, Q;
    int Wp;        // padded width: 32 x waves
    int RB, nseg, items;
    int remap;
    const float* ps;  // fused epilogue (EPI): y = act(y * ps[k] + pb[k]); either may be NULL
    const float* pb;
    int act;
};

// PD: raw ring slots (PD - 1 rows in flight ahead of the one being split).
// NTS: non-temporal output stores.  EPI: fused eval-BN affine + activation.
// V (variant bits, autotune candidates): 1 = B fragments held in VGPRs for the kernel's
// lifetime (no per-step LDS weight reads; 3 waves per SIMD), 2 = direct stores from the
// accumulators (each lane's float4 = 4 consecutive pixels of one channel; two 64-byte
// runs per channel per row) instead of the LDS transpose.  LDS read traffic slows the
// DMA stream of this kernel (r02 probe: +18 ds_read_b128 per row ~ +3 % time).
// DBG (diagnostic builds only, -DPO2Q_ROWS_DIAG, PO2Q_ROWSF_DEBUG; timing only, outputs
// wrong): 1 = no split and no MFMAs, 2 = no transpose (stores straight from registers),
// 4 = no x DMAs, 8 = stores dropped (still issued, out of range).  Product: DBG = 0.
template <int PD, bool EPI, int NTS, int V = 0, int DBG = 0>
__global__ __launch_bounds__(448, (V & 1) ? 3 : 4) void conv_rowsf(const float* __restrict__ x, const uint4* __restrict__ wpk,
                                                     const float* __restrict__ scale_p,
                                                     const float* __restrict__ bias, float* __restrict__ y,
                                                     RowsFArgs a) {
    static_assert(PD >= 2 && PD <= 6, "raw ring slots");
    constexpr int KS = 2;  // k-steps per tap row: (s=0 | s=1) x 16 channels, (s=2 | zero slot)
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int rawslot = 16 * a.Wp * 4;
    uint4* wl = reinterpret_cast<uint4*>(lds);
    unsigned char* raw = lds + kFWBytes;                                  // PD slots [16][Wp] fp32
    unsigned char* slab = raw + PD * rawslot + wave * (3 * kFPlane);      // this wave's planes
    const int zero_off = kFWC * 16 * 2;

    for (int e = tid; e < 3 * KS * 64; e += blockDim.x) wl[e] = wpk[e];
    if (lane < 3) *reinterpret_cast<uint4*>(slab + lane * kFPlane + zero_off) = make_uint4(0u, 0u, 0u, 0u);
    float bk = bias ? bias[lane & 15] : 0.0f;
    float eps_ = (EPI && a.ps) ? a.ps[lane & 15] : 1.0f;
    float epb_ = (EPI && a.pb) ? a.pb[lane & 15] : 0.0f;
    const float scale = *scale_p;
    bf16x8 bwr[(V & 1) ? 3 * KS : 1];
    if constexpr (V & 1) {
#pragma unroll
        for (int f = 0; f < 3 * KS; ++f) {
            bwr[f] = __builtin_bit_cast(bf16x8, wpk[f * 64 + lane]);
            asm volatile("s_waitcnt vmcnt(0)" : "+v"(bwr[f]));
        }
    }
    // the parameter loads land here (tied), not at their first use inside the row loop
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(bk), "+v"(eps_), "+v"(epb_));
    auto outv = [&](float accv) __attribute__((always_inline)) {
        const float v = accv * scale + bk;
        if constexpr (EPI)
            return epi_act(v * eps_ + epb_, a.act);
        else
            return v;
    };
    __syncthreads();

    int blk = blockIdx.x;
    if (a.remap) blk = (blk & 7) * (int)(gridDim.x >> 3) + (blk >> 3);
    if (blk >= a.items) return;  // block-uniform
    const int seg = blk % a.nseg;
    const int n = blk / a.nseg;
    const int p0 = seg * a.RB;
    const int rbe = min(a.RB, a.P - p0);
    const int nrows = rbe + 2;  // halo rows p0-1 .. p0+rbe
    const int q0 = wave * kFSW;

    // ---- DMA: this wave's 2 instructions of a row; lane l of instruction i (global index
    // 2w + i) -> element e = 64(2w + i) + l of the row's 16 x Wp/4 float4: channel
    // e / (Wp/4), float4 column e % (Wp/4).  Columns >= W read out of range (zeros).
    const int HW = a.H * a.W;
    const __amdgpu_buffer_rsrc_t rs = rows_rsrc(x + (int64_t)n * 16 * HW, 16 * HW * 4);
    const int W4 = a.Wp >> 2;
    uint32_t vi[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int e = 64 * (2 * wave + i) + lane;
        const int c = e / W4, q = 4 * (e - c * W4);
        vi[i] = q < a.W ? ((uint32_t)c * (uint32_t)HW + (uint32_t)q) * 4u : 0x7fffffffu;
    }
    const uint32_t raw_lds = (uint32_t)(uintptr_t)raw;
    auto load_row = [&](int sl, int j) __attribute__((always_inline)) {
        const int h = p0 - 1 + j;
        const bool hok = j < nrows && h >= 0 && h < a.H;
        const uint32_t roff = (uint32_t)(hok ? h : 0) * (uint32_t)a.W * 4u;
        const uint32_t base = raw_lds + (uint32_t)(sl * rawslot) + (uint32_t)(2 * wave) * 1024u;
#pragma unroll
        for (int i = 0; i < 2; ++i)
            rows_dma16<false>(rs, (hok && vi[i] != 0x7fffffffu && !(DBG & 4)) ? vi[i] + roff : 0x7fffffffu, 0u,
                              base + i * 1024u);
    };

    // ---- split: lane -> (column sc of the strip, channel octet so); halo: lane < 32 ->
    // (side, channel), read from the neighbours' columns of the raw row (zero outside)
    const int sc = lane & 31, so = lane >> 5;
    const int rd0 = (so * 8) * (a.Wp * 4) + (q0 + sc) * 4;
    const int wa_i = x_addr<16>(sc + 1, so);
    const int hside = (lane >> 4) & 1, hch = lane & 15;
    const int hq = hside ? q0 + kFSW : q0 - 1;
    const bool h_ok = lane < 32 && hq >= 0 && hq < a.W;
    const int rd_h = hch * (a.Wp * 4) + (h_ok ? hq : 0) * 4;
    const int wa_h = x_addr<16>(hside ? kFWC - 1 : 0, hch >> 3) + (hch & 7) * 2;

    // ---- A fragment addresses (plane-relative) per (group, k-step)
    int aoff[2][KS];
    {
        const int p = lane & 15, g = lane >> 4;
#pragma unroll
        for (int grp = 0; grp < 2; ++grp) {
            aoff[grp][0] = x_addr<16>(16 * grp + p + (g >> 1), g & 1);
            aoff[grp][1] = (g < 2) ? x_addr<16>(16 * grp + p + 2, g & 1) : zero_off;
        }
    }
    const int PQ = a.P * a.Q;
    const __amdgpu_buffer_rsrc_t ry = rows_rsrc(y + (int64_t)n * 16 * PQ, 16 * PQ * 4);
    constexpr int ST = 2;  // stores per step (issued every step; dropped ones out of range)
    // vm ops issued after this wave's DMAs of row j (step j - PD + 1, after its barrier)
    // until the wait of step j: that step's ST stores, then 2 DMAs + ST stores per step
    constexpr int VMW = ST + (PD - 2) * (2 + ST);

    floatx4 acc[3][2];
#pragma unroll
    for (int sl = 0; sl < 3; ++sl)
#pragma unroll
        for (int grp = 0; grp < 2; ++grp) acc[sl][grp] = floatx4{0.f, 0.f, 0.f, 0.f};

    auto step = [&](auto S_, int j) __attribute__((always_inline)) {
        constexpr int S6 = decltype(S_)::value;
        constexpr int S = S6 % 3;  // accumulator rotation
        const int RS = (6 % PD == 0) ? S6 % PD : j % PD;
        const unsigned char* rw = raw + RS * rawslot;
        rows_wait<VMW>();                 // this wave's part of row j has landed
        __builtin_amdgcn_s_barrier();     // ... and every other wave's; row j - 1 is split
        // refill the slot of row j - 1 with row j - 1 + PD
        {
            const int jn = j - 1 + PD;
            load_row((6 % PD == 0) ? (S6 + PD - 1) % PD : jn % PD, jn);
        }
        // split row j: own 32 columns x 16 channels, and the two halo columns
        if constexpr (!(DBG & 1)) {
            uint32_t b8[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) b8[e] = *reinterpret_cast<const uint32_t*>(rw + rd0 + e * (a.Wp * 4));
            uint32_t hb = *reinterpret_cast<const uint32_t*>(rw + rd_h);
            hb = h_ok ? hb : 0u;
            uint4 hi, mid, lo;
            split3(b8, hi, mid, lo);
            *reinterpret_cast<uint4*>(slab + wa_i) = hi;
            *reinterpret_cast<uint4*>(slab + kFPlane + wa_i) = mid;
            *reinterpret_cast<uint4*>(slab + 2 * kFPlane + wa_i) = lo;
            if (lane < 32) {
                uint16_t h16, m16, l16;
                split1(hb, h16, m16, l16);
                *reinterpret_cast<uint16_t*>(slab + wa_h) = h16;
                *reinterpret_cast<uint16_t*>(slab + kFPlane + wa_h) = m16;
                *reinterpret_cast<uint16_t*>(slab + 2 * kFPlane + wa_h) = l16;
            }
        }
        // MFMAs: halo row j feeds output halo-index j+1 (r=0), j (r=1), j-1 (r=2)
        constexpr int SL[3] = {(S + 1) % 3, S, (S + 2) % 3};
#pragma unroll
        for (int ks = 0; ks < KS && !(DBG & 1); ++ks) {
            bf16x8 af[3][2];
#pragma unroll
            for (int pl = 0; pl < 3; ++pl)
#pragma unroll
                for (int grp = 0; grp < 2; ++grp)
                    af[pl][grp] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(slab + pl * kFPlane + aoff[grp][ks]));
#pragma unroll
            for (int rr = 0; rr < 3; ++rr) {
                const bf16x8 bw = (V & 1) ? bwr[(V & 1) ? rr * KS + ks : 0]
                                          : __builtin_bit_cast(bf16x8, wl[(rr * KS + ks) * 64 + lane]);
#pragma unroll
                for (int pl = 0; pl < 3; ++pl)
#pragma unroll
                    for (int grp = 0; grp < 2; ++grp)
                        acc[SL[rr]][grp] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[pl][grp], bw, acc[SL[rr]][grp], 0, 0, 0);
            }
        }
        // output halo-index j-1 (row p0 + j - 2) is complete: transpose the [16][32] fp32
        // row through the planes' first 2 KiB (their A fragments are read: this wave's LDS
        // ops run in order) so each store writes 8 whole 128-byte channel runs; 16-byte
        // blocks XOR-swizzled by channel.  Plane 0's zero slot lies in that window.
        constexpr int D = (S + 2) % 3;
        const int o = p0 + j - 2;
        const bool orow = j >= 2 && o < p0 + rbe;
        if constexpr ((V & 2) || (DBG & 2)) {
            const uint32_t yk = (uint32_t)(lane & 15) * (uint32_t)PQ + (uint32_t)(orow ? o : 0) * a.Q;
#pragma unroll
            for (int grp = 0; grp < 2; ++grp) {
                const int q = q0 + 16 * grp + 4 * (lane >> 4);
                floatx4 v;
                v[0] = outv(acc[D][grp][0]);
                v[1] = outv(acc[D][grp][1]);
                v[2] = outv(acc[D][grp][2]);
                v[3] = outv(acc[D][grp][3]);
                rows_store<(NTS & 1) != 0>(ry, (orow && q < a.Q && !(DBG & 8)) ? (yk + (uint32_t)q) * 4u : 0x7fffffffu, v);
            }
        } else {
            const int ch = lane & 15, g = lane >> 4;
#pragma unroll
            for (int grp = 0; grp < 2; ++grp) {
                floatx4 v;
                v[0] = outv(acc[D][grp][0]);
                v[1] = outv(acc[D][grp][1]);
                v[2] = outv(acc[D][grp][2]);
                v[3] = outv(acc[D][grp][3]);
                *reinterpret_cast<floatx4*>(slab + ch * 128 + 16 * ((4 * grp + g) ^ (ch & 7))) = v;
            }
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int c = (lane >> 3) + 8 * i, b = lane & 7;
                const floatx4 v = *reinterpret_cast<const floatx4*>(slab + c * 128 + 16 * (b ^ (c & 7)));
                const int q = q0 + 4 * b;
                const uint32_t yo = (uint32_t)c * (uint32_t)PQ + (uint32_t)(orow ? o : 0) * a.Q + q;
                rows_store<(NTS & 1) != 0>(ry, (orow && q < a.Q && !(DBG & 8)) ? yo * 4u : 0x7fffffffu, v);
            }
            if (lane == 0) *reinterpret_cast<uint4*>(slab + zero_off) = make_uint4(0u, 0u, 0u, 0u);
        }
#pragma unroll
        for (int grp = 0; grp < 2; ++grp) acc[D][grp] = floatx4{0.f, 0.f, 0.f, 0.f};
    };

    {
        // rows 0 .. PD-2, each followed by ST dropped stores: the steady-state count holds
        // from the first step on
        const floatx4 z = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int r = 0; r < PD - 1; ++r) {
            load_row(r, r);
#pragma unroll
            for (int i = 0; i < ST; ++i) rows_store<(NTS & 1) != 0>(ry, 0x7fffffffu, z);
        }
    }
    // every wave runs the same steps (block-uniform nrows): the barriers pair up; steps
    // past nrows DMA nothing (out of range) and store nothing
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
static size_t rowsf_lds(int waves, int pd) {
    return (size_t)kFWBytes + (size_t)pd * 16 * (32 * waves) * 4 + (size_t)waves * 3 * kFPlane;
}

void rowsf_candidates(const ConvPlan& b, int mode, int bits, int fsr, std::vector<PlanCand>& out) {
    if (mode == 0 || b.groups != 1) return;
    if (bits < 1 || bits > 16) return;
    const long lo = (long)fsr - (1L << (bits - 1)), hi = (long)fsr - 1;
    if (lo < -126 || hi > 127) return;  // +-2^e must be a normal bf16
    if (b.R != 3 || b.S != 3 || b.sh != 1 || b.sw != 1 || b.ph != 1 || b.pw != 1 || b.dh != 1 || b.dw != 1) return;
    if (b.C != 16 || b.K != 16 || b.Q % 4 != 0) return;
    const int waves = (b.W + kFSW - 1) / kFSW;
    if (waves < 1 || waves > 7) return;  // 448-thread blocks (launch bounds)
    if ((int64_t)16 * b.H * b.W * 4 >= (1LL << 31) || (int64_t)16 * b.P * b.Q * 4 >= (1LL << 31)) return;
    ConvPlan p = b;
    p.kind = KIND_BF16X3_ROWS;
    p.vrx = 4;  // full-row blocks
    p.CC = 16; p.NT = 1; p.NJ = 2; p.TQ = 32 * waves;
    p.steps = 2; p.nchunks = 1; p.kblocks = 1; p.taps = 9;
    p.PS = 0; p.MI = 0; p.nts = 0;
    p.dma_d0 = p.dma_nck = p.dma_ni = p.dma_nw = p.dma_waves = p.dma_ov = 0;
    p.HH = 0; p.WW = p.WWp = kFWC;
    p.SB = 32;
    p.plane = kFPlane;
    p.packed_floats = (int64_t)3 * p.steps * p.NT * 64 * 4;
    p.tilesQ = 1;
    for (int pd : {3, 4}) {
        ConvPlan q = p;
        q.pd = pd;
        q.lds_bytes = rowsf_lds(waves, pd);
        // blocks per CU: VGPR budget (4 waves per SIMD) and LDS
        const int per_cu = std::min(12 / waves, (int)(160 * 1024 / q.lds_bytes));
        if (per_cu < 1) continue;
        const int slots = 256 * per_cu;
        std::vector<std::pair<double, int>> rbs;
        for (int rb = 4; rb <= p.P; ++rb) {
            const int nseg = (p.P + rb - 1) / rb;
            if (rb != (p.P + nseg - 1) / nseg) continue;
            const int64_t items = (int64_t)p.N * nseg;
            if (items > INT_MAX / 2) continue;
            rbs.push_back({(double)((items + slots - 1) / slots) * (rb + 2), rb});
        }
        std::sort(rbs.begin(), rbs.end());
        // variants (plan field PS = V): 0 plain, 1 VGPR weights, 2 direct stores, 3 both
        for (int v : {0, 1, 2, 3})
            for (int nts : {0, 1})
                for (int i = 0; i < (int)rbs.size() && i < 2; ++i) {
                    ConvPlan c = q;
                    c.TP = rbs[i].second;
                    c.tilesP = (p.P + c.TP - 1) / c.TP;
                    c.blocks = ((int64_t)p.N * c.tilesP + 7) / 8 * 8;
                    c.nts = nts;
                    c.PS = v;
                    out.push_back({0.89 + 0.001 * i + 0.002 * nts + 0.003 * (pd - 3) + 0.0005 * v, c});
                }
    }
}

hipError_t launch_conv_rowsf(const ConvPlan& p, const float* x, const uint16_t* packed, const float* scale,
                             const float* bias, float* y, hipStream_t s, const float* ps, const float* pb, int act,
                             bool epi) {
    RowsFArgs a;
    a.N = p.N; a.H = p.H; a.W = p.W; a.P = p.P; a.Q = p.Q;
    const int waves = p.TQ / 32;
    a.Wp = p.TQ;
    a.RB = p.TP; a.nseg = p.tilesP;
    a.items = p.N * p.tilesP;
    a.remap = (p.blocks % 8 == 0) ? 1 : 0;
    a.ps = ps; a.pb = pb; a.act = act;
    if (p.vrx != 4 || p.C != 16 || p.K != 16 || waves < 1 || waves > 7) return hipErrorInvalidValue;
#ifdef PO2Q_ROWS_DIAG
    if (const char* dv = getenv("PO2Q_ROWSF_DEBUG")) {
        const int dbg = atoi(dv);
#define PO2Q_RFD(v)                                                                                             \
    if (dbg == v && p.pd == 4 && p.nts == 1 && p.PS == 1 && !epi) {                                            \
        hipLaunchKernelGGL((conv_rowsf<4, false, 1, 1, v>), dim3((unsigned)p.blocks), dim3(64 * waves), p.lds_bytes, \
                           s, x, reinterpret_cast<const uint4*>(packed), scale, bias, y, a);                  \
        return hipGetLastError();                                                                              \
    }
        PO2Q_RFD(1) PO2Q_RFD(2) PO2Q_RFD(3) PO2Q_RFD(4) PO2Q_RFD(8) PO2Q_RFD(5) PO2Q_RFD(10) PO2Q_RFD(11)
#undef PO2Q_RFD
    }
#endif
#define PO2Q_RF(d, e, nt, v)                                                                                  \
    if (p.pd == d && epi == e && p.nts == nt && p.PS == v) {                                                   \
        hipLaunchKernelGGL((conv_rowsf<d, e, nt, v>), dim3((unsigned)p.blocks), dim3(64 * waves), p.lds_bytes, s, \
                           x, reinterpret_cast<const uint4*>(packed), scale, bias, y, a);                     \
        return hipGetLastError();                                                                              \
    }
#define PO2Q_RFV(d, e, nt) PO2Q_RF(d, e, nt, 0) PO2Q_RF(d, e, nt, 1) PO2Q_RF(d, e, nt, 2) PO2Q_RF(d, e, nt, 3)
    PO2Q_RFV(3, false, 0) PO2Q_RFV(3, false, 1) PO2Q_RFV(4, false, 0) PO2Q_RFV(4, false, 1)
    PO2Q_RFV(3, true, 0) PO2Q_RFV(3, true, 1) PO2Q_RFV(4, true, 0) PO2Q_RFV(4, true, 1)
#undef PO2Q_RFV
#undef PO2Q_RF
    return hipErrorInvalidValue;
}

}  // namespace po2q
