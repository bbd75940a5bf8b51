// bf16x3 row-streaming conv for 3x3 / stride 1 / pad 1 layers with C = 16 or 32
// (ResNet56 stages 1 and 2: 35 of its 56 quantized convs, ~75 % of the forward).
//
// Same arithmetic as po2q_conv_x3.hip (exact +-2^e bf16 weights x exact 3-way bf16
// split of the fp32 activations, fp32 accumulation on v_mfma_f32_16x16x32_bf16;
// reference: QuantizedConv2d.forward, models/quantized_conv.py:32-38), different
// work decomposition, built for HBM streaming without block-wide barriers:
//
//   * one WAVE owns one work item = (image, column strip of 32 (C = 16) or 16
//     (C = 32) output columns, segment of RB output rows) and marches down it one
//     input (halo) row at a time;
//   * per halo row, LDS-DMA (`buffer_load_dwordx4 ... lds`, 1 KiB per instruction,
//     no VGPRs) brings the strip's interior [C][columns] fp32 block into a 2-slot raw
//     ring of the wave's LDS slab, plus one dword DMA for the two halo columns; the
//     buffer range check supplies the zero padding;
//   * a split pass reads 8 channels of one column per lane (ds_read_b32), splits
//     them exactly into hi / mid / lo bf16 and writes the three [column][C] planes
//     (ds_write_b128); A fragments are read back from the planes and feed the THREE
//     output rows the halo row contributes to (row reuse: every activation is
//     loaded, split and read once per tap row, not once per tap);
//   * three accumulator slots rotate over output rows (loop unrolled by 6: slots
//     mod 3, raw slots mod 2 -- every index static); a completed output row is
//     scaled, biased and stored from the accumulators (C = 16: transposed through
//     LDS so each store instruction writes 8 whole 128-byte channel runs);
//   * the DMA of halo row j+2 is issued right after row j is split, so two rows are
//     in flight per wave (16 / 12 waves per CU); every global access of the loop is
//     inline asm with one exact `s_waitcnt vmcnt` per step (hipcc's own bookkeeping
//     falls back to vmcnt(0) at the loop header, i.e. waits for every store);
//   * no block-wide barrier after the one-time weight staging: the slab is
//     wave-private and a wave's LDS operations complete in issue order.
//   * weights: the B fragments of all (tap row r, k-step, 16-channel tile) live in
//     LDS for the block's lifetime (6 KiB for 16->16, 18 KiB for 32->32).
//
// k-steps per tap row: C = 16: two -- k = (s=0 | s=1) x 16 channels, then (s=2 | zero
// slot); C = 32: three -- k = 32 channels of tap s.
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

struct RowsArgs {
    int N, C, H, W, K, P, Q;
    int RB, nseg, nstrip, items;
    int plane;     // bytes per split plane (halo columns x C x 2 + zero slot + pad)
    int slab;      // bytes per wave slab: 3 planes + 2 raw slots
    int w_bytes;   // weight fragment bytes at the start of LDS
    int remap;     // XCD-aware block order (gridDim.x % 8 == 0)
    const float* ps;  // fused epilogue (EPI): y = act(y * ps[k] + pb[k]); either may be NULL
    const float* pb;
    int act;
};

constexpr int kRawInterior = 2048;             // [C][strip columns] fp32 (C x SW = 512 floats)
constexpr int kRawSlot = kRawInterior + 256;   // + the halo dwords (64 lanes)

// DBG (diagnostic builds only, -DPO2Q_ROWS_DIAG): timing ablation bits -- 1 no MFMA,
// 2 no split (raw bits to the planes), 4 no x loads, 8 no stores, 16 nt stores, 32 no
// halo-column DMA.  Product:
// DBG = 0.  NTS (plan field nts, autotune candidates): bit 0 = output stores, bit 1 = x
// loads (LDS-DMA) with the non-temporal policy.
// The fused residual add lives in the full-row kernel (po2q_conv_rowsf.hip: residual rows
// DMA'd into LDS behind the counted row wait); this kernel leaves it to the elementwise pass.
// PD: halo rows in flight per wave (raw ring slots).  What bounds this kernel is the
// bytes in flight per CU, and those live in LDS (the DMA targets): PD = 2 at 16 waves per
// CU keeps 32 rows (64 KiB) in flight, PD = 6 at 8 waves 48 rows.
template <int CC, int NT, int DBG = 0, bool EPI = false, int NTS = 0, int PD = 2>
__global__ __launch_bounds__(kThreads, CC == 16 ? 4 : 3) void conv_rows(const float* __restrict__ x,
                                                                     const uint4* __restrict__ wpk,
                                                                     const float* __restrict__ scale_p,
                                                                     const float* __restrict__ bias,
                                                                     float* __restrict__ y, RowsArgs a) {
    static_assert(PD >= 2 && PD <= 6, "raw ring slots");
    constexpr int NG = 32 / CC;       // 16-pixel groups per wave
    constexpr int SW = 16 * NG;       // strip width (output columns)
    constexpr int WC = SW + 2;        // halo columns
    constexpr int KS = CC == 16 ? 2 : 3;
    constexpr int NFR = 3 * KS * NT;  // B fragments (64 lanes x 16 B each)
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar loop control

    // ---- one-time staging: weight fragments (block), zero slots (per wave)
    uint4* wl = reinterpret_cast<uint4*>(lds);
    for (int e = tid; e < NFR * 64; e += kThreads) wl[e] = wpk[e];
    unsigned char* slab = lds + a.w_bytes + wave * a.slab;
    unsigned char* raw = slab + 3 * a.plane;  // PD raw slots
    const int zero_off = WC * CC * 2;
    if (lane < 3) *reinterpret_cast<uint4*>(slab + lane * a.plane + zero_off) = make_uint4(0u, 0u, 0u, 0u);
    float bk[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        const int k = nt * 16 + (lane & 15);
        bk[nt] = bias ? bias[k] : 0.0f;
    }
    const float scale = *scale_p;
    float eps_[NT], epb_[NT];  // fused epilogue: per-lane channel affine
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        const int k = nt * 16 + (lane & 15);
        eps_[nt] = (EPI && a.ps) ? a.ps[k] : 1.0f;
        epb_[nt] = (EPI && a.pb) ? a.pb[k] : 0.0f;
    }
    // the bias loads land here (tied), not at their first use inside the row loop,
    // where hipcc would otherwise wait for vmcnt(0) -- every prefetch and store
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) asm volatile("s_waitcnt vmcnt(0)" : "+v"(bk[nt]), "+v"(eps_[nt]), "+v"(epb_[nt]));
    // scaled accumulator -> output value (+ fused eval-BN affine and activation)
    auto outv = [&](float accv, int nt) __attribute__((always_inline)) {
        const float v = accv * scale + bk[nt];
        if constexpr (EPI)
            return epi_act(v * eps_[nt] + epb_[nt], a.act);
        else
            return v;
    };
    __syncthreads();

    // XCD-aware block order: dispatch puts block b on XCD b % 8; the blocks one XCD
    // runs take consecutive items, so strips that share halo columns (and segments
    // that share halo rows) meet in the same L2
    int blk = blockIdx.x;
    if (a.remap) blk = (blk & 7) * (int)(gridDim.x >> 3) + (blk >> 3);
    const int item = blk * (kThreads / 64) + wave;
    if (item >= a.items) return;
    const int strip = item % a.nstrip;
    const int t0 = item / a.nstrip;
    const int seg = t0 % a.nseg;
    const int n = t0 / a.nseg;
    const int q0 = strip * SW;
    const int p0 = seg * a.RB;
    const int rbe = min(a.RB, a.P - p0);
    const int nrows = rbe + 2;  // halo rows p0-1 .. p0+rbe

    // ---- DMA descriptors.  Interior: instruction i, lane l -> 16 B = columns
    // 4*cb .. 4*cb+3 of channel cl + CPI*i; lane-linear landing makes the raw slot a
    // row-major [C][SW] fp32 block.  Halo: lane l < 2C -> (side, channel).
    const int HW = a.H * a.W;
    const uint32_t cstride = (uint32_t)HW * 4u;
    const __amdgpu_buffer_rsrc_t rs = [&] {
        const uintptr_t bp = reinterpret_cast<uintptr_t>(x + (int64_t)n * a.C * HW);
        const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)bp);
        const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(bp >> 32));
        void* b = reinterpret_cast<void*>(((uintptr_t)hi << 32) | lo);
        return __builtin_amdgcn_make_buffer_rsrc(b, (short)0, a.C * HW * 4, 0x00020000);  // planner: < 2^31
    }();
    constexpr int LPC = SW / 4;    // lanes per channel row
    constexpr int CPI = 64 / LPC;  // channels per DMA instruction
    const int cb = lane % LPC, cl = lane / LPC;
    const int gq4 = q0 + 4 * cb;
    const bool qi_ok = gq4 < a.W;  // W % 4 == 0 (planner): a 4-column block is all in or all out
    const uint32_t vi0 = (uint32_t)cl * cstride + (uint32_t)gq4 * 4u;
    const uint32_t soff1 = (uint32_t)CPI * cstride;
    const bool hl = lane < 2 * CC;
    const int hside = lane / CC, hch = lane % CC;
    const int gqh = hside ? q0 + SW : q0 - 1;
    const bool qh_ok = hl && gqh >= 0 && gqh < a.W;
    const uint32_t vh0 = (uint32_t)hch * cstride + (uint32_t)gqh * 4u;
    const uint32_t raw_lds = (uint32_t)(uintptr_t)raw;  // LDS byte address of raw slot 0

    // ---- split pass mapping: lane -> (strip column sc, channel octet so), 8 channels
    const int sc = lane % SW, so = lane / SW;
    const int rd0 = (so * 8) * (SW * 4) + sc * 4;  // raw byte offset of channel 8*so, column sc
    const int wa_i = x_addr<CC>(sc + 1, so);
    const int wa_h = x_addr<CC>(hside ? WC - 1 : 0, hch >> 3) + (hch & 7) * 2;

    // ---- A fragment addresses (plane-relative) per (group, k-step)
    int aoff[NG][KS];
    {
        const int p = lane & 15, g = lane >> 4;
#pragma unroll
        for (int grp = 0; grp < NG; ++grp) {
            if constexpr (CC == 16) {
                aoff[grp][0] = x_addr<16>(16 * grp + p + (g >> 1), g & 1);
                aoff[grp][1] = (g < 2) ? x_addr<16>(16 * grp + p + 2, g & 1) : zero_off;
            } else {
#pragma unroll
                for (int s = 0; s < 3; ++s) aoff[grp][s] = x_addr<32>(16 * grp + p + s, g);
            }
        }
    }

    // 3 DMAs per halo row into raw slot `sl`
    auto load_row = [&](int sl, int j) __attribute__((always_inline)) {
        const int h = p0 - 1 + j;
        const bool hok = j < nrows && h >= 0 && h < a.H;
        const uint32_t roff = (uint32_t)(hok ? h : 0) * (uint32_t)a.W * 4u;
        const uint32_t vo = (hok && qi_ok) ? vi0 + roff : 0x7fffffffu;
        const uint32_t base = raw_lds + (uint32_t)(sl * kRawSlot);
        rows_dma16<(NTS & 2) != 0>(rs, vo, 0u, base);
        rows_dma16<(NTS & 2) != 0>(rs, vo, soff1, base + 1024u);
        const uint32_t voh = (hok && qh_ok) ? vh0 + roff : 0x7fffffffu;
        if constexpr (!(DBG & 32)) rows_dma4<(NTS & 2) != 0>(rs, voh, base + (uint32_t)kRawInterior);
    };
    constexpr int ST = NG * NT;      // epilogue stores per step (issued every step)
    // vm ops issued after a row's DMAs (end of step j - PD: DMA, MFMAs, ST stores) until
    // the wait of step j: that step's stores, then per step in between 3 DMAs + ST stores
    constexpr int VMW = ST + (PD - 1) * (3 + ST);
    // output descriptor (per image): dropped stores take an out-of-range voffset
    const __amdgpu_buffer_rsrc_t ry = [&] {
        const uintptr_t yp = reinterpret_cast<uintptr_t>(y + (int64_t)n * a.K * a.P * a.Q);
        const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)yp);
        const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(yp >> 32));
        void* yb = reinterpret_cast<void*>(((uintptr_t)hi << 32) | lo);
        return __builtin_amdgcn_make_buffer_rsrc(yb, (short)0, a.K * a.P * a.Q * 4, 0x00020000);
    }();

    floatx4 acc[3][NG][NT];
#pragma unroll
    for (int sl = 0; sl < 3; ++sl)
#pragma unroll
        for (int grp = 0; grp < NG; ++grp)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) acc[sl][grp][nt] = floatx4{0.f, 0.f, 0.f, 0.f};

    const int PQ = a.P * a.Q;

    // one halo row j (j % 6 == S6): wait for its DMAs, split raw -> planes, DMA row j+2
    // into the raw slot just split, MFMAs, store output row j-1.
    auto step = [&](auto S_, int j) __attribute__((always_inline)) {
        constexpr int S6 = decltype(S_)::value;
        constexpr int S = S6 % 3;   // accumulator rotation
        // raw slot of row j (static when PD divides the 6-step unroll)
        const int RS = (6 % PD == 0) ? S6 % PD : j % PD;
        const unsigned char* rw = raw + RS * kRawSlot;
        if constexpr (!(DBG & 4)) rows_wait<VMW>();
        // split + write this halo row into the planes
        {
            uint32_t b8[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) b8[e] = *reinterpret_cast<const uint32_t*>(rw + rd0 + e * (SW * 4));
            uint4 hi, mid, lo;
            if constexpr (DBG & 2) {
                hi = make_uint4(b8[0], b8[1], b8[2], b8[3]);
                mid = lo = make_uint4(b8[4], b8[5], b8[6], b8[7]);
            } else {
                split3(b8, hi, mid, lo);
            }
            *reinterpret_cast<uint4*>(slab + wa_i) = hi;
            *reinterpret_cast<uint4*>(slab + a.plane + wa_i) = mid;
            *reinterpret_cast<uint4*>(slab + 2 * a.plane + wa_i) = lo;
            if (hl) {
                uint16_t h16, m16, l16;
                split1(*reinterpret_cast<const uint32_t*>(rw + kRawInterior + 4 * lane), h16, m16, l16);
                *reinterpret_cast<uint16_t*>(slab + wa_h) = h16;
                *reinterpret_cast<uint16_t*>(slab + a.plane + wa_h) = m16;
                *reinterpret_cast<uint16_t*>(slab + 2 * a.plane + wa_h) = l16;
            }
        }
        // prefetch halo row j+PD into the raw slot just split
        if constexpr (!(DBG & 4)) load_row(RS, j + PD);
        // MFMAs: halo row j feeds output halo-index j+1 (r=0), j (r=1), j-1 (r=2)
        constexpr int SL[3] = {(S + 1) % 3, S, (S + 2) % 3};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            bf16x8 af[3][NG];
#pragma unroll
            for (int pl = 0; pl < 3; ++pl)
#pragma unroll
                for (int grp = 0; grp < NG; ++grp)
                    af[pl][grp] = __builtin_bit_cast(
                        bf16x8, *reinterpret_cast<const uint4*>(slab + pl * a.plane + aoff[grp][ks]));
#pragma unroll
            for (int rr = 0; rr < 3; ++rr) {
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) {
                    const bf16x8 bw = __builtin_bit_cast(bf16x8, wl[((rr * KS + ks) * NT + nt) * 64 + lane]);
#pragma unroll
                    for (int pl = 0; pl < 3; ++pl)
#pragma unroll
                        for (int grp = 0; grp < NG; ++grp)
                            if constexpr (DBG & 1) {  // keep the operands alive, skip the matrix core
                                acc[SL[rr]][grp][nt][0] += __builtin_bit_cast(float, (uint32_t)af[pl][grp][0]) +
                                                           __builtin_bit_cast(float, (uint32_t)bw[0]);
                            } else {
                                acc[SL[rr]][grp][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                                    af[pl][grp], bw, acc[SL[rr]][grp][nt], 0, 0, 0);
                            }
                }
            }
        }
        // output halo-index j-1 (row p0 + j - 2) is complete
        constexpr int D = (S + 2) % 3;
        const int o = p0 + j - 2;
        const bool orow = j >= 2 && o < p0 + rbe;
        if constexpr (!(DBG & 8) && NG == 2) {
            // 32-column strips: transpose the [16 channels][32 columns] fp32 row through
            // the planes' first 2 KiB (their A fragments are read: this wave's LDS ops
            // run in order) so every store instruction writes 8 whole 128-byte channel
            // runs; 16-byte blocks XOR-swizzled by channel.  Plane 0's zero slot lies in
            // that window and is re-zeroed after.
            const int ch = lane & 15, g = lane >> 4;
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
#pragma unroll
                for (int grp = 0; grp < NG; ++grp) {
                    floatx4 v;
                    v[0] = outv(acc[D][grp][nt][0], nt);
                    v[1] = outv(acc[D][grp][nt][1], nt);
                    v[2] = outv(acc[D][grp][nt][2], nt);
                    v[3] = outv(acc[D][grp][nt][3], nt);
                    *reinterpret_cast<floatx4*>(slab + ch * 128 + 16 * ((4 * grp + g) ^ (ch & 7))) = v;
                }
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const int c = (lane >> 3) + 8 * i, b = lane & 7;
                    const floatx4 v = *reinterpret_cast<const floatx4*>(slab + c * 128 + 16 * (b ^ (c & 7)));
                    const int q = q0 + 4 * b;
                    const uint32_t yo = (uint32_t)(nt * 16 + c) * (uint32_t)PQ + (uint32_t)(orow ? o : 0) * a.Q + q;
                    rows_store<(NTS & 1) != 0 || (DBG & 16) != 0>(ry, (orow && q < a.Q) ? yo * 4u : 0x7fffffffu, v);
                }
            }
            if (lane == 0) *reinterpret_cast<uint4*>(slab + zero_off) = make_uint4(0u, 0u, 0u, 0u);
        } else if constexpr (!(DBG & 8)) {
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
                const uint32_t yk = (uint32_t)(nt * 16 + (lane & 15)) * (uint32_t)PQ + (uint32_t)(orow ? o : 0) * a.Q;
#pragma unroll
                for (int grp = 0; grp < NG; ++grp) {
                    const int q = q0 + 16 * grp + 4 * (lane >> 4);
                    floatx4 v;
                    v[0] = outv(acc[D][grp][nt][0], nt);
                    v[1] = outv(acc[D][grp][nt][1], nt);
                    v[2] = outv(acc[D][grp][nt][2], nt);
                    v[3] = outv(acc[D][grp][nt][3], nt);
                    rows_store<(NTS & 1) != 0 || (DBG & 16) != 0>(ry, (orow && q < a.Q) ? (yk + (uint32_t)q) * 4u : 0x7fffffffu, v);
                }
            }
        }
#pragma unroll
        for (int grp = 0; grp < NG; ++grp)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) acc[D][grp][nt] = floatx4{0.f, 0.f, 0.f, 0.f};
    };

    if constexpr (!(DBG & 4)) {
        // rows 0 .. PD-1, each followed by ST dropped stores: the steady-state count of
        // vm ops between a row's DMAs and its split holds from the first step on
        const floatx4 z = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int r = 0; r < PD; ++r) {
            load_row(r, r);
            if constexpr (!(DBG & 8))
#pragma unroll
                for (int i = 0; i < ST; ++i) rows_store<(NTS & 1) != 0 || (DBG & 16) != 0>(ry, 0x7fffffffu, z);
        }
    }
    // steps past nrows DMA zeros (out of range) and store nothing: at most 5 per item
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
static int cdivr(int a, int b) { return (a + b - 1) / b; }

// output channels across the block's waves (po2q_conv_rowsk.hip: C = K in {32, 64})
void rowsk_candidates(const ConvPlan& b, int mode, int bits, int fsr, std::vector<PlanCand>& out);
hipError_t launch_conv_rowsk(const ConvPlan& p, const float* x, const uint16_t* packed, const float* scale,
                             const float* bias, float* y, hipStream_t s, const float* ps, const float* pb,
                             int act, bool epi, const WQuant& q);
// full-row blocks (po2q_conv_rowsf.hip: C = K = 16, plan vrx = 4)
void rowsf_candidates(const ConvPlan& b, int mode, int bits, int fsr, std::vector<PlanCand>& out);
hipError_t launch_conv_rowsf(const ConvPlan& p, const float* x, const uint16_t* packed, const float* scale,
                             const float* bias, float* y, hipStream_t s, const float* ps, const float* pb, int act,
                             bool epi, const WQuant& q);
bool rowsf_res_ok(const ConvPlan& p);
hipError_t launch_conv_rowsf_res(const ConvPlan& p, const float* x, const uint16_t* packed, const float* scale,
                                 const float* bias, float* y, const float* ps, const float* pb, const float* res,
                                 int act, hipStream_t s, const WQuant& q);

// stride-2 full-row blocks (po2q_conv_rows2.hip: 3x3 s2 16 -> 32, plan vrx = 5); launch_conv_rows2
// is declared in po2q_internal.h
void rows2_candidates(const ConvPlan& b, int mode, int bits, int fsr, std::vector<PlanCand>& out);

void rows_candidates(const ConvPlan& base, int mode, int bits, int fsr, std::vector<PlanCand>& out) {
    const ConvPlan& b = base;
    rowsk_candidates(base, mode, bits, fsr, out);
    rowsf_candidates(base, mode, bits, fsr, out);
    rows2_candidates(base, mode, bits, fsr, out);
    if (mode == 0 || b.groups != 1) return;
    if (bits < 1 || bits > 16) return;
    const long lo = (long)fsr - (1L << (bits - 1)), hi = (long)fsr - 1;
    if (lo < -126 || hi > 127) return;  // +-2^e must be a normal bf16
    if (b.R != 3 || b.S != 3 || b.sh != 1 || b.sw != 1 || b.ph != 1 || b.pw != 1 || b.dh != 1 || b.dw != 1) return;
    // (C, K) with a non-spilling instantiation
    if (!((b.C == 16 && b.K == 16) || (b.C == 32 && (b.K == 16 || b.K == 32)))) return;
    if (b.Q % 4 != 0) return;  // float4 epilogue; with stride 1 / pad 1, W == Q: 16-byte DMAs
    if ((int64_t)b.C * b.H * b.W * 4 >= (1LL << 31)) return;  // 32-bit buffer offsets per image
    if ((int64_t)b.K * b.P * b.Q * 4 >= (1LL << 31)) return;
    ConvPlan p = b;
    p.kind = KIND_BF16X3_ROWS;
    p.CC = b.C;
    p.NT = b.K / 16;
    p.NJ = 32 / p.CC;
    p.TQ = 16 * p.NJ;
    p.steps = p.CC == 16 ? 2 : 3;
    p.nchunks = 1;
    p.kblocks = 1;
    p.taps = 9;
    p.vrx = 0; p.PS = 0; p.MI = 0; p.pd = 2;
    p.dma_d0 = p.dma_nck = p.dma_ni = p.dma_nw = p.dma_waves = p.dma_ov = 0;
    p.HH = 0; p.WW = p.WWp = p.TQ + 2;
    p.SB = 2 * p.CC;
    p.plane = p.WW * p.SB + 32;
    const int w_bytes = 3 * p.steps * p.NT * 1024;
    p.packed_floats = (int64_t)3 * p.steps * p.NT * 64 * 4;
    p.tilesQ = cdivr(p.Q, p.TQ);
    const int vgpr_waves = p.CC == 16 ? 16 : 12;  // per CU: 4 / 3 per SIMD (launch bounds)
    // prefetch depth (raw ring slots): C = 16 also 3 and 6 -- fewer waves per CU (LDS),
    // more rows in flight
    std::vector<int> pds = {2};
    if (p.CC == 16) pds = {2, 3, 6};
    for (int pd : pds) {
        ConvPlan q = p;
        q.pd = pd;
        q.lds_bytes = (size_t)w_bytes + 4 * (3 * (size_t)p.plane + (size_t)pd * kRawSlot);
        const int blocks_cu = std::min(vgpr_waves / 4, (int)(160 * 1024 / q.lds_bytes));
        if (blocks_cu < 1) continue;
        // rows per segment: minimise (rounds of resident waves) x (halo rows per item)
        const int slots = 256 * 4 * blocks_cu;
        std::vector<std::pair<double, int>> rbs;
        for (int rb = 8; rb <= p.P; ++rb) {
            const int nseg = cdivr(p.P, rb);
            if (rb != cdivr(p.P, nseg)) continue;  // one RB per segment count
            const int64_t items = (int64_t)p.N * nseg * p.tilesQ;
            if (items > INT_MAX / 2) continue;
            const int64_t rounds = (items + slots - 1) / slots;
            rbs.push_back({(double)rounds * (rb + 2), rb});
        }
        std::sort(rbs.begin(), rbs.end());
        // plain and non-temporal output stores (interleaved A/B on stage 1: 4-5 % faster on
        // some boxes, r01_v14); non-temporal x loads measured slower for this walk
        // (r02: 0.41 vs 0.36 ms), so none.  The autotuner decides.
        for (int nts : {0, 1})
            for (int i = 0; i < (int)rbs.size() && i < (pd == 2 ? 3 : 2); ++i) {
                ConvPlan c = q;
                c.TP = rbs[i].second;
                c.tilesP = cdivr(p.P, c.TP);
                const int64_t items = (int64_t)p.N * c.tilesP * c.tilesQ;
                c.blocks = ((items + 3) / 4 + 7) / 8 * 8;  // whole XCD rounds (extra waves exit at once)
                c.nts = nts;
                // cost comparable with the other bf16x3 planners (their cost ~ 1.0 + overheads)
                out.push_back({0.9 + 0.005 * nts + 0.001 * i + (pd == 2 ? 0.0 : 0.002 * pd), c});
            }
    }
}

template <int CC, int NT, int DBG = 0, bool EPI = false, int NTS = 0, int PD = 2>
static hipError_t launch_rows_t(const ConvPlan& p, const float* x, const uint16_t* packed, const float* scale,
                                const float* bias, float* y, hipStream_t s, const float* ps = nullptr,
                                const float* pb = nullptr, int act = 0) {
    RowsArgs a;
    a.N = p.N; a.C = p.C; a.H = p.H; a.W = p.W; a.K = p.K; a.P = p.P; a.Q = p.Q;
    a.RB = p.TP; a.nseg = p.tilesP; a.nstrip = p.tilesQ;
    a.items = p.N * p.tilesP * p.tilesQ;
    a.plane = p.plane;
    a.slab = 3 * p.plane + PD * kRawSlot;
    if (p.pd != PD) return hipErrorInvalidValue;
    a.w_bytes = 3 * p.steps * p.NT * 1024;
    a.remap = (p.blocks % 8 == 0) ? 1 : 0;
    a.ps = ps;
    a.pb = pb;
    a.act = act;
    hipLaunchKernelGGL((conv_rows<CC, NT, DBG, EPI, NTS, PD>), dim3((unsigned)p.blocks), dim3(kThreads), p.lds_bytes, s, x,
                       reinterpret_cast<const uint4*>(packed), scale, bias, y, a);
    return hipGetLastError();
}

// (CC, NT) x nts -> instantiation; the planner only emits the variants that fit their
// register budget without spilling
template <bool EPI>
static hipError_t rows_dispatch(const ConvPlan& p, const float* x, const uint16_t* packed, const float* scale,
                                const float* bias, float* y, hipStream_t s, const float* ps, const float* pb,
                                int act) {
#define PO2Q_ROWS_NTS(cc, nt, d)                                                                                \
    if (p.CC == cc && p.NT == nt && p.pd == d) {                                                                 \
        if (p.nts == 1) return launch_rows_t<cc, nt, 0, EPI, 1, d>(p, x, packed, scale, bias, y, s, ps, pb, act); \
        if (p.nts == 0) return launch_rows_t<cc, nt, 0, EPI, 0, d>(p, x, packed, scale, bias, y, s, ps, pb, act); \
        return hipErrorInvalidValue;                                                                             \
    }
    PO2Q_ROWS_NTS(16, 1, 2) PO2Q_ROWS_NTS(16, 1, 3) PO2Q_ROWS_NTS(16, 1, 6)
    PO2Q_ROWS_NTS(32, 1, 2) PO2Q_ROWS_NTS(32, 2, 2)
#undef PO2Q_ROWS_NTS
    return hipErrorInvalidValue;
}

hipError_t launch_conv_bf16x3_rows(const ConvPlan& p, const float* x, const uint16_t* packed, const float* scale,
                                   const float* bias, float* y, hipStream_t s, const WQuant& q) {
    if (p.vrx == 5) return launch_conv_rows2(p, x, bias, y, s, nullptr, nullptr, 0, false, q);
    if (p.vrx == 4) return launch_conv_rowsf(p, x, packed, scale, bias, y, s, nullptr, nullptr, 0, false, q);
    if (p.vrx) return launch_conv_rowsk(p, x, packed, scale, bias, y, s, nullptr, nullptr, 0, false, q);
    if (p.fp) return hipErrorInvalidValue;  // fused weight staging: full-row / C = 64 plans only
#ifdef PO2Q_ROWS_DIAG
    const char* dbg = getenv("PO2Q_ROWS_DEBUG");  // timing ablation (outputs are wrong)
    if (dbg && p.CC == 32 && p.NT == 2) {
        switch (atoi(dbg)) {
#define PO2Q_ROWS_CASE(d) \
    case d: return launch_rows_t<32, 2, d>(p, x, packed, scale, bias, y, s);
            PO2Q_ROWS_CASE(1) PO2Q_ROWS_CASE(2) PO2Q_ROWS_CASE(4) PO2Q_ROWS_CASE(8) PO2Q_ROWS_CASE(12)
            PO2Q_ROWS_CASE(3) PO2Q_ROWS_CASE(14)
#undef PO2Q_ROWS_CASE
            default: break;
        }
    }
    if (dbg && p.CC == 16 && p.NT == 1) {
        switch (atoi(dbg)) {
#define PO2Q_ROWS_CASE(d) \
    case d: return launch_rows_t<16, 1, d>(p, x, packed, scale, bias, y, s);
            PO2Q_ROWS_CASE(1) PO2Q_ROWS_CASE(2) PO2Q_ROWS_CASE(3) PO2Q_ROWS_CASE(4) PO2Q_ROWS_CASE(5)
            PO2Q_ROWS_CASE(6) PO2Q_ROWS_CASE(7) PO2Q_ROWS_CASE(8) PO2Q_ROWS_CASE(9) PO2Q_ROWS_CASE(12)
            PO2Q_ROWS_CASE(13) PO2Q_ROWS_CASE(14) PO2Q_ROWS_CASE(15) PO2Q_ROWS_CASE(16) PO2Q_ROWS_CASE(20)
            PO2Q_ROWS_CASE(32) PO2Q_ROWS_CASE(35) PO2Q_ROWS_CASE(19) PO2Q_ROWS_CASE(51) PO2Q_ROWS_CASE(48)
#undef PO2Q_ROWS_CASE
            default: break;
        }
    }
#endif
    // the planner only emits the variants that fit their register budget without spilling
    return rows_dispatch<false>(p, x, packed, scale, bias, y, s, nullptr, nullptr, 0);
}

}  // namespace po2q

namespace po2q {

hipError_t launch_conv_bf16x3_rows_epi(const ConvPlan& p, const float* x, const uint16_t* packed,
                                       const float* scale, const float* bias, float* y, const float* ps,
                                       const float* pb, int act, hipStream_t s, const WQuant& q) {
    if (p.vrx == 5) return launch_conv_rows2(p, x, bias, y, s, ps, pb, act, true, q);
    if (p.vrx == 4) return launch_conv_rowsf(p, x, packed, scale, bias, y, s, ps, pb, act, true, q);
    if (p.vrx) return launch_conv_rowsk(p, x, packed, scale, bias, y, s, ps, pb, act, true, q);
    if (p.fp) return hipErrorInvalidValue;
    return rows_dispatch<true>(p, x, packed, scale, bias, y, s, ps, pb, act);
}

// The residual add inside the kernel (po2q_epi.h): the full-row plans (C = K = 16 / 32,
// residual rows DMA'd into LDS behind the row wait), the C = K = 32 loader-wave plans and
// every C = K = 64 plan (as its TT sibling).
// The per-wave row kernel leaves it to the elementwise pass.
bool rows_res_ok(const ConvPlan& p) { return rowsf_res_ok(p) || rowsk_res_ok(p); }

hipError_t launch_conv_rows_res(const ConvPlan& p, const float* x, const uint16_t* packed, const float* scale,
                                const float* bias, float* y, const float* ps, const float* pb, const float* res,
                                int act, hipStream_t s, const WQuant& q) {
    if (rowsf_res_ok(p)) return launch_conv_rowsf_res(p, x, packed, scale, bias, y, ps, pb, res, act, s, q);
    if (rowsk_res_ok(p)) return launch_conv_rowsk_res(p, x, packed, scale, bias, y, ps, pb, res, act, s, q);
    return hipErrorInvalidValue;
}

}  // namespace po2q
