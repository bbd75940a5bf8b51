// bf16x3 full-row-block conv for 3x3 / stride 1 / pad 1 with C = K = 16 or 32 (ResNet56
// stages 1 and 2: 35 of its 56 quantized convs).
//
// Same arithmetic as the other bf16x3 kernels (exact +-2^e bf16 weights x exact 3-way bf16
// split of the fp32 activations, fp32 accumulation on v_mfma_f32_16x16x32_bf16; reference:
// QuantizedConv2d.forward, models/quantized_conv.py:32-38) and the same per-wave compute as
// po2q_conv_rows.hip (a wave owns SW = 512 / C output columns and all K = C output
// channels, row reuse over the 3 tap rows, 3 rotating accumulator slots).  What changes is
// the walk:
//
//   * one BLOCK owns (image, segment of RB output rows) across the WHOLE width: wave w of
//     the W/SW waves owns columns SW*w .. SW*w + SW - 1;
//   * per halo row the block LDS-DMAs the row's C channel runs (C x W fp32, one 4W-byte
//     run per channel) into a raw ring slot [C][Wp]; every wave issues 2 of the 1-KiB
//     instructions, so the memory system sees whole-row runs, not 128-byte strips (r01
//     probe, stage 2: full-row walks 0.16-0.18 ms vs 0.19-0.21 for 32-column strips);
//   * no halo-column DMA: a wave reads its two halo columns straight from the neighbours'
//     part of the shared raw row (r02 probe: the per-strip halo dword DMA cost ~5 % of the
//     stage-1 layer; tools/copy_probe.hip mode 2);
//   * one s_barrier per row: each wave waits for its own DMAs (exact vmcnt), the barrier
//     makes the whole row visible, and the slot of the previous row (split by every wave
//     before this barrier) is refilled right after it -- PD - 1 rows stay in flight.
//   * RES (fused residual add): each wave DMAs the residual of its own strip for the row
//     it will store PD - 1 steps later into a wave-private ring, behind the same wait.
//   * FP (fused weight staging, plan field fp): the block reduces max|w| and quantizes +
//     packs its B fragments itself (po2q_quant_dev.h wq_*), so the layer is ONE launch --
//     the reference's quantize-then-conv (quantized_conv.py:35-36) without the pack kernel.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdlib>
#include <type_traits>
#include <vector>

#include "po2q_epi.h"
#include "po2q_internal.h"
#include "po2q_quant_dev.h"
#include "po2q_rows_dev.h"
#include "po2q_x3_dev.h"

namespace po2q {

namespace {
template <int CC> constexpr int kFSW = 512 / CC;                      // output columns per wave
template <int CC> constexpr int kFWC = kFSW<CC> + 2;                  // halo columns per wave
template <int CC> constexpr int kFPlane = kFWC<CC> * CC * 2 + 32;     // bf16 plane (+ zero slot, pad)
template <int CC> constexpr int kFKS = CC == 16 ? 2 : 3;              // k-steps per tap row
template <int CC> constexpr int kFWBytes = 3 * kFKS<CC> * (CC / 16) * 1024;  // B fragments
constexpr int kFResSlot = 2048;  // residual of one wave's strip and row: [C][SW] fp32
constexpr int64_t kFusedStageMax = 65536;  // fp plans: every block re-reads the weight from L2
}  // namespace

struct RowsFArgs {
    int N, H, W, P, Q;
    int Wp;        // padded width: SW x waves
    int RB, nseg, items;
    int remap;
    const float* ps;  // fused epilogue (EPI): y = act(y * ps[k] + pb[k] (+ res)); either may be NULL
    const float* pb;
    int act;
    const float* res;  // RES: residual [N, K, P, Q]
    WQuant q;          // FP: raw weights + quantizer parameters
};

// PD: raw ring slots (PD - 1 rows in flight ahead of the one being split).
// NTS bit 0: non-temporal output stores, bit 1: non-temporal x loads.  EPI: fused eval-BN
// affine + activation.
// V (variant bits, autotune candidates): 1 = B fragments held in VGPRs for the kernel's
// lifetime (no per-step LDS weight reads; C = 32: 72 VGPRs of weights, 2 waves per
// SIMD, one block per CU), 2 = direct stores from the
// accumulators (C = 16; each lane's float4 = 4 consecutive pixels of one channel, two
// 64-byte runs per channel and row) instead of the LDS transpose.  C = 32 always stores
// directly (a wave's strip is 16 columns: 64-byte runs either way).
// DBG (diagnostic builds only, -DPO2Q_ROWS_DIAG, PO2Q_ROWSF_DEBUG; timing only, outputs
// wrong): 1 = no split and no MFMAs, 2 = no transpose (stores straight from registers),
// 4 = no x DMAs, 8 = stores dropped (still issued, out of range).  Product: DBG = 0.
template <int CC, int PD, bool EPI, int NTS, int V = 0, bool RES = false, int DBG = 0, bool FP = false>
__global__ __launch_bounds__(448, (CC == 32 && (V & 1)) ? 2 : 4) void conv_rowsf(const float* __restrict__ x, const uint4* __restrict__ wpk,
                                                     const float* __restrict__ scale_p,
                                                     const float* __restrict__ bias, float* __restrict__ y,
                                                     RowsFArgs a) {
    static_assert(CC == 16 || CC == 32, "C = K = 16 or 32");
    static_assert(PD >= 2 && PD <= 6, "raw ring slots");
    static_assert(CC == 16 || V <= 1, "C = 32: direct stores");
    static_assert(!RES || EPI, "the residual add is part of the fused epilogue");
    constexpr int SW = kFSW<CC>, WC = kFWC<CC>, PL = kFPlane<CC>, KS = kFKS<CC>;
    constexpr int NG = SW / 16;   // 16-pixel groups per wave
    constexpr int NT = CC / 16;   // 16-channel output tiles (K = C)
    constexpr bool TR = CC == 16 && !(V & 2) && !(DBG & 2);  // stores through the LDS transpose
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nw = (int)(blockDim.x >> 6);
    const int rawslot = CC * a.Wp * 4;
    uint4* wl = reinterpret_cast<uint4*>(lds);
    unsigned char* raw = lds + kFWBytes<CC>;                           // PD slots [C][Wp] fp32
    unsigned char* slab = raw + PD * rawslot + wave * (3 * PL);        // this wave's planes
    unsigned char* resr = raw + PD * rawslot + nw * (3 * PL) + wave * (PD * kFResSlot);  // RES ring
    const int zero_off = WC * CC * 2;

    // per-lane epilogue parameters and (V & 1) weight fragments: set by the staging below,
    // after the first row DMAs are on their way
    float scale = 1.0f;
    bool fin = true;
    float bk[NT], eps_[NT], epb_[NT];
    bf16x8 bwr[(V & 1) ? 3 * KS * NT : 1];
    // accumulator -> output value; with RES the activation follows the residual add
    auto outv = [&](float accv, int nt) __attribute__((always_inline)) {
        const float v = accv * scale + bk[nt];
        if constexpr (EPI && RES)
            return v * eps_[nt] + epb_[nt];
        else if constexpr (EPI)
            return epi_act(v * eps_[nt] + epb_[nt], a.act);
        else
            return v;
    };

    int blk = blockIdx.x;
    if (a.remap) blk = (blk & 7) * (int)(gridDim.x >> 3) + (blk >> 3);
    if (blk >= a.items) return;  // block-uniform
    const int seg = blk % a.nseg;
    const int n = blk / a.nseg;
    const int p0 = seg * a.RB;
    const int rbe = min(a.RB, a.P - p0);
    const int nrows = rbe + 2;  // halo rows p0-1 .. p0+rbe
    const int q0 = wave * SW;

    // ---- DMA: this wave's 2 instructions of a row; lane l of instruction i (global index
    // 2w + i) -> element e = 64(2w + i) + l of the row's C x Wp/4 float4: channel
    // e / (Wp/4), float4 column e % (Wp/4).  Columns >= W read out of range (zeros).
    const int HW = a.H * a.W;
    const __amdgpu_buffer_rsrc_t rs = rows_rsrc(x + (int64_t)n * CC * HW, CC * HW * 4);
    const int W4 = a.Wp >> 2;
    uint32_t vi[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int e = 64 * (2 * wave + i) + lane;
        const int c = e / W4, q = 4 * (e - c * W4);
        vi[i] = q < a.W ? ((uint32_t)c * (uint32_t)HW + (uint32_t)q) * 4u : 0x7fffffffu;
    }
    const uint32_t raw_lds = (uint32_t)(uintptr_t)raw;
    const int PQ = a.P * a.Q;
    // RES: this wave's strip of one residual row, lane-linear [C][SW] fp32 (2 KiB, two
    // instructions): lane l of instruction i -> channel (64i + l) / (SW/4), float4 column
    const __amdgpu_buffer_rsrc_t rres = rows_rsrc(RES ? a.res + (int64_t)n * CC * PQ : x, RES ? CC * PQ * 4 : 4);
    uint32_t vr[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int e = 64 * i + lane;
        const int c = e / (SW / 4), q = q0 + 4 * (e % (SW / 4));
        vr[i] = q < a.Q ? ((uint32_t)c * (uint32_t)PQ + (uint32_t)q) * 4u : 0x7fffffffu;
    }
    const uint32_t res_lds = (uint32_t)(uintptr_t)resr;
    // row jn's DMAs (and with RES the residual of the row stored at step jn) into slot sl
    auto load_row = [&](int sl, int jn) __attribute__((always_inline)) {
        const int h = p0 - 1 + jn;
        const bool hok = jn < nrows && h >= 0 && h < a.H;
        const uint32_t roff = (uint32_t)(hok ? h : 0) * (uint32_t)a.W * 4u;
        const uint32_t base = raw_lds + (uint32_t)(sl * rawslot) + (uint32_t)(2 * wave) * 1024u;
#pragma unroll
        for (int i = 0; i < 2; ++i)
            rows_dma16<(NTS & 2) != 0>(rs, (hok && vi[i] != 0x7fffffffu && !(DBG & 4)) ? vi[i] + roff : 0x7fffffffu, 0u,
                              base + i * 1024u);
        if constexpr (RES) {
            const int o = jn - 2;  // output row index within the segment
            const bool ook = jn >= 2 && o < rbe;
            const uint32_t ooff = (uint32_t)(ook ? p0 + o : 0) * (uint32_t)a.Q * 4u;
#pragma unroll
            for (int i = 0; i < 2; ++i)
                rows_dma16<false>(rres, (ook && vr[i] != 0x7fffffffu) ? vr[i] + ooff : 0x7fffffffu, 0u,
                                  res_lds + (uint32_t)(sl * kFResSlot) + i * 1024u);
        }
    };

    // ---- split: lane -> (column sc of the strip, channel octet so); halo: lane < 2C ->
    // (side, channel), read from the neighbours' columns of the raw row (zero outside)
    const int sc = lane % SW, so = lane / SW;
    const int rd0 = (so * 8) * (a.Wp * 4) + (q0 + sc) * 4;
    const int wa_i = x_addr<CC>(sc + 1, so);
    const int hside = (lane / CC) & 1, hch = lane % CC;
    const int hq = hside ? q0 + SW : q0 - 1;
    const bool h_ok = lane < 2 * CC && hq >= 0 && hq < a.W;
    const int rd_h = hch * (a.Wp * 4) + (h_ok ? hq : 0) * 4;
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
    const __amdgpu_buffer_rsrc_t ry = rows_rsrc(y + (int64_t)n * CC * PQ, CC * PQ * 4);
    constexpr int ST = NG * NT;       // stores per step (issued every step; dropped ones out of range)
    constexpr int LD = RES ? 4 : 2;   // DMAs per step
    // vm ops issued after this wave's DMAs for step j (issued in step j - PD + 1, after its
    // barrier) until the wait of step j: that step's ST stores, then LD DMAs + ST stores
    // per step in between
    constexpr int VMW = ST + (PD - 2) * (LD + ST);

    floatx4 acc[3][NG][NT];
#pragma unroll
    for (int sl = 0; sl < 3; ++sl)
#pragma unroll
        for (int grp = 0; grp < NG; ++grp)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) acc[sl][grp][nt] = floatx4{0.f, 0.f, 0.f, 0.f};

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
        // split row j: own SW columns x C channels, and the two halo columns
        if constexpr (!(DBG & 1)) {
            uint32_t b8[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) b8[e] = *reinterpret_cast<const uint32_t*>(rw + rd0 + e * (a.Wp * 4));
            uint32_t hb = *reinterpret_cast<const uint32_t*>(rw + rd_h);
            hb = h_ok ? hb : 0u;
            uint4 hi, mid, lo;
            split3(b8, hi, mid, lo);
            *reinterpret_cast<uint4*>(slab + wa_i) = hi;
            *reinterpret_cast<uint4*>(slab + PL + wa_i) = mid;
            *reinterpret_cast<uint4*>(slab + 2 * PL + wa_i) = lo;
            if (lane < 2 * CC) {
                uint16_t h16, m16, l16;
                split1(hb, h16, m16, l16);
                *reinterpret_cast<uint16_t*>(slab + wa_h) = h16;
                *reinterpret_cast<uint16_t*>(slab + PL + wa_h) = m16;
                *reinterpret_cast<uint16_t*>(slab + 2 * PL + wa_h) = l16;
            }
        }
        // MFMAs: halo row j feeds output halo-index j+1 (r=0), j (r=1), j-1 (r=2)
        constexpr int SL[3] = {(S + 1) % 3, S, (S + 2) % 3};
#pragma unroll
        for (int ks = 0; ks < KS && !(DBG & 1); ++ks) {
            bf16x8 af[3][NG];
#pragma unroll
            for (int pl = 0; pl < 3; ++pl)
#pragma unroll
                for (int grp = 0; grp < NG; ++grp)
                    af[pl][grp] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(slab + pl * PL + aoff[grp][ks]));
#pragma unroll
            for (int rr = 0; rr < 3; ++rr) {
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) {
                    const bf16x8 bw = (V & 1) ? bwr[(V & 1) ? (rr * KS + ks) * NT + nt : 0]
                                              : __builtin_bit_cast(bf16x8, wl[((rr * KS + ks) * NT + nt) * 64 + lane]);
#pragma unroll
                    for (int pl = 0; pl < 3; ++pl)
#pragma unroll
                        for (int grp = 0; grp < NG; ++grp)
                            acc[SL[rr]][grp][nt] =
                                __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[pl][grp], bw, acc[SL[rr]][grp][nt], 0, 0, 0);
                }
            }
        }
        // output halo-index j-1 (row p0 + j - 2) is complete
        constexpr int D = (S + 2) % 3;
        const int o = p0 + j - 2;
        const bool orow = j >= 2 && o < p0 + rbe;
        const unsigned char* rres_row = resr + RS * kFResSlot;  // RES: the slot loaded with row j
        if constexpr (!TR) {
            // lane: channel nt*16 + (lane & 15), pixels 4 (lane >> 4) .. +3 of group grp
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
                const int ck = nt * 16 + (lane & 15);
                const uint32_t yk = (uint32_t)ck * (uint32_t)PQ + (uint32_t)(orow ? o : 0) * a.Q;
#pragma unroll
                for (int grp = 0; grp < NG; ++grp) {
                    const int ql = 16 * grp + 4 * (lane >> 4);  // strip column
                    const int q = q0 + ql;
                    floatx4 v;
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = outv(acc[D][grp][nt][e], nt);
                    if constexpr (RES) {
                        const floatx4 r = *reinterpret_cast<const floatx4*>(rres_row + ck * (SW * 4) + 4 * ql);
#pragma unroll
                        for (int e = 0; e < 4; ++e) v[e] = epi_act(v[e] + r[e], a.act);
                    }
                    rows_store<(NTS & 1) != 0>(ry, (orow && q < a.Q && !(DBG & 8)) ? (yk + (uint32_t)q) * 4u : 0x7fffffffu, v);
                }
            }
        } else {
            // C = 16: transpose the [16][32] fp32 row through the planes' first 2 KiB (their
            // A fragments are read: this wave's LDS ops run in order) so each store writes 8
            // whole 128-byte channel runs; 16-byte blocks XOR-swizzled by channel.  Plane 0's
            // zero slot lies in that window and is re-zeroed after.
            const int ch = lane & 15, g = lane >> 4;
#pragma unroll
            for (int grp = 0; grp < NG; ++grp) {
                floatx4 v;
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = outv(acc[D][grp][0][e], 0);
                *reinterpret_cast<floatx4*>(slab + ch * 128 + 16 * ((4 * grp + g) ^ (ch & 7))) = v;
            }
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int c = (lane >> 3) + 8 * i, b = lane & 7;
                floatx4 v = *reinterpret_cast<const floatx4*>(slab + c * 128 + 16 * (b ^ (c & 7)));
                if constexpr (RES) {
                    const floatx4 r = *reinterpret_cast<const floatx4*>(rres_row + c * 128 + 16 * b);
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = epi_act(v[e] + r[e], a.act);
                }
                const int q = q0 + 4 * b;
                const uint32_t yo = (uint32_t)c * (uint32_t)PQ + (uint32_t)(orow ? o : 0) * a.Q + q;
                rows_store<(NTS & 1) != 0>(ry, (orow && q < a.Q && !(DBG & 8)) ? yo * 4u : 0x7fffffffu, v);
            }
            if (lane == 0) *reinterpret_cast<uint4*>(slab + zero_off) = make_uint4(0u, 0u, 0u, 0u);
        }
#pragma unroll
        for (int grp = 0; grp < NG; ++grp)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) acc[D][grp][nt] = floatx4{0.f, 0.f, 0.f, 0.f};
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
    // ---- weights, staged while those DMAs fly: fused quantize + pack (FP; scratch in wave
    // 0's planes, free until its first split) or the pre-packed workspace.  Their loads are
    // compiler-visible and younger than the DMAs: the waits hipcc places for them are
    // stricter than the counted row waits, never looser.
    {
        unsigned* red = reinterpret_cast<unsigned*>(raw + PD * rawslot);
        unsigned* thr = red + 16;
        if constexpr (FP) {
            scale = wq_prologue(a.q, thr, red, nw, fin);
            // the block packs every fragment once into wl (V & 1 then copies its own into VGPRs)
            wq_pack_rows_lds<CC>(a.q, CC, CC, NT, KS, scale, fin, thr, wl, 3 * KS * NT);
        } else {
            for (int e = tid; e < 3 * KS * NT * 64; e += blockDim.x) wl[e] = wpk[e];
            scale = *scale_p;
        }
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
            const int k = nt * 16 + (lane & 15);
            bk[nt] = bias ? bias[k] : 0.0f;
            eps_[nt] = (EPI && a.ps) ? a.ps[k] : 1.0f;
            epb_[nt] = (EPI && a.pb) ? a.pb[k] : 0.0f;
        }
        if constexpr (V & 1) {
#pragma unroll
            for (int f = 0; f < 3 * KS * NT; ++f) {
                if constexpr (FP)
                    bwr[f] = __builtin_bit_cast(bf16x8, wl[f * 64 + lane]);
                else
                    bwr[f] = __builtin_bit_cast(bf16x8, wpk[f * 64 + lane]);
            }
        }
        // every staged value lands here (tied), not at a first use inside the row loop
        // (that wait would be a vmcnt(0) behind the loop's DMAs and stores)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) asm volatile("" : "+v"(bk[nt]), "+v"(eps_[nt]), "+v"(epb_[nt]));
        if constexpr (V & 1) {
#pragma unroll
            for (int f = 0; f < 3 * KS * NT; ++f) asm volatile("" : "+v"(bwr[f]));
        }
        // zero slots (own planes; outside the scratch words), then wl and the scratch reads
        // complete block-wide: wave 0's planes are first written after step 0's barrier
        if (lane < 3) *reinterpret_cast<uint4*>(slab + lane * PL + zero_off) = make_uint4(0u, 0u, 0u, 0u);
        __syncthreads();
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
static size_t rowsf_lds(int C, int waves, int pd) {
    const int plane = C == 16 ? kFPlane<16> : kFPlane<32>;
    const int wbytes = C == 16 ? kFWBytes<16> : kFWBytes<32>;
    const int sw = 512 / C;
    return (size_t)wbytes + (size_t)pd * C * (sw * waves) * 4 + (size_t)waves * 3 * plane;
}
static size_t rowsf_res_lds(const ConvPlan& p) { return p.lds_bytes + (size_t)(p.TQ / (512 / p.C)) * p.pd * kFResSlot; }

void rowsf_candidates(const ConvPlan& b, int mode, int bits, int fsr, std::vector<PlanCand>& out) {
    if (mode == 0 || b.groups != 1) return;
    if (bits < 1 || bits > 16) return;
    const long lo = (long)fsr - (1L << (bits - 1)), hi = (long)fsr - 1;
    if (lo < -126 || hi > 127) return;  // +-2^e must be a normal bf16
    if (b.R != 3 || b.S != 3 || b.sh != 1 || b.sw != 1 || b.ph != 1 || b.pw != 1 || b.dh != 1 || b.dw != 1) return;
    if (!((b.C == 16 && b.K == 16) || (b.C == 32 && b.K == 32)) || b.Q % 4 != 0) return;
    const int sw = 512 / b.C;
    const int waves = (b.W + sw - 1) / sw;
    if (waves < 1 || waves > 7) return;  // 448-thread blocks (launch bounds)
    if ((int64_t)b.C * b.H * b.W * 4 >= (1LL << 31) || (int64_t)b.K * b.P * b.Q * 4 >= (1LL << 31)) return;
    ConvPlan p = b;
    p.kind = KIND_BF16X3_ROWS;
    p.vrx = 4;  // full-row blocks
    p.CC = b.C; p.NT = b.K / 16; p.NJ = sw / 16; p.TQ = sw * waves;
    p.steps = b.C == 16 ? 2 : 3; p.nchunks = 1; p.kblocks = 1; p.taps = 9;
    p.PS = 0; p.MI = 0; p.nts = 0;
    p.dma_d0 = p.dma_nck = p.dma_ni = p.dma_nw = p.dma_waves = p.dma_ov = 0;
    p.HH = 0; p.WW = p.WWp = sw + 2;
    p.SB = 2 * b.C;
    p.plane = b.C == 16 ? kFPlane<16> : kFPlane<32>;
    p.packed_floats = (int64_t)3 * p.steps * p.NT * 64 * 4;
    p.tilesQ = 1;
    // variants (plan field PS = V): C = 16: 0 plain, 1 VGPR weights, 2 direct stores;
    // C = 32: 0 only.  nts: see the candidate loop
    const std::vector<int> vs = b.C == 16 ? std::vector<int>{0, 1, 2} : std::vector<int>{0, 1};
    for (int pd : {3, 4, 2}) {
        if (b.C == 16 && pd == 2) continue;
        ConvPlan q = p;
        q.pd = pd;
        q.lds_bytes = rowsf_lds(b.C, waves, pd);
        for (int v : vs) {
            // blocks per CU: VGPR budget (4 waves per SIMD; C = 32 with VGPR weights 2) and LDS
            const int per_cu = std::min((b.C == 32 && (v & 1) ? 8 : 16) / waves, (int)(160 * 1024 / q.lds_bytes));
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
            // nts: bit 0 non-temporal stores (C = 16 only: slower with 64-byte runs), bit 1
            // non-temporal x loads (the pair kernel's best mode, r02_pair_nt.log)
            for (int nts : {0, 1, 2, 3}) {
                if (nts && v == 2) continue;
                if (b.C == 32 ? (nts & 1) != 0 : nts == 2) continue;
                for (int i = 0; i < (int)rbs.size() && i < 2; ++i) {
                    ConvPlan c = q;
                    c.TP = rbs[i].second;
                    c.tilesP = (p.P + c.TP - 1) / c.TP;
                    c.blocks = ((int64_t)p.N * c.tilesP + 7) / 8 * 8;
                    c.nts = nts;
                    c.PS = v;
                    // fused weight staging first (one launch), then the pre-packed form
                    for (int fp : {1, 0}) {
                        if (fp && (int64_t)b.K * b.C * 9 > kFusedStageMax) continue;
                        c.fp = fp;
                        out.push_back({0.889 + 0.001 * fp + 0.001 * i + 0.002 * nts + 0.003 * (pd - 3) + 0.0005 * v, c});
                    }
                }
            }
        }
    }
}

template <int CC, int PD, bool EPI, int NTS, int V, bool RES = false, int DBG = 0>
static hipError_t launch_rowsf_t(const ConvPlan& p, const RowsFArgs& a, const float* x, const uint16_t* packed,
                                 const float* scale, const float* bias, float* y, hipStream_t s) {
    const int waves = p.TQ / kFSW<CC>;
    const size_t lds = RES ? rowsf_res_lds(p) : p.lds_bytes;
    if (p.fp) {
        if (!a.q.w) return hipErrorInvalidValue;
        hipLaunchKernelGGL((conv_rowsf<CC, PD, EPI, NTS, V, RES, DBG, true>), dim3((unsigned)p.blocks), dim3(64 * waves),
                           lds, s, x, reinterpret_cast<const uint4*>(packed), scale, bias, y, a);
    } else {
        hipLaunchKernelGGL((conv_rowsf<CC, PD, EPI, NTS, V, RES, DBG>), dim3((unsigned)p.blocks), dim3(64 * waves), lds,
                           s, x, reinterpret_cast<const uint4*>(packed), scale, bias, y, a);
    }
    return hipGetLastError();
}

static bool rowsf_plan_ok(const ConvPlan& p) {
    if (p.kind != KIND_BF16X3_ROWS || p.vrx != 4 || !((p.C == 16 && p.K == 16) || (p.C == 32 && p.K == 32))) return false;
    const int waves = p.TQ / (512 / p.C);
    return waves >= 1 && waves <= 7 && p.TQ == waves * (512 / p.C);
}

static RowsFArgs rowsf_args(const ConvPlan& p, const float* ps, const float* pb, int act, const float* res,
                            const WQuant& q) {
    RowsFArgs a;
    a.N = p.N; a.H = p.H; a.W = p.W; a.P = p.P; a.Q = p.Q;
    a.Wp = p.TQ;
    a.RB = p.TP; a.nseg = p.tilesP;
    a.items = p.N * p.tilesP;
    a.remap = (p.blocks % 8 == 0) ? 1 : 0;
    a.ps = ps; a.pb = pb; a.act = act; a.res = res;
    a.q = q;
    return a;
}

hipError_t launch_conv_rowsf(const ConvPlan& p, const float* x, const uint16_t* packed, const float* scale,
                             const float* bias, float* y, hipStream_t s, const float* ps, const float* pb, int act,
                             bool epi, const WQuant& q) {
    if (!rowsf_plan_ok(p)) return hipErrorInvalidValue;
    const RowsFArgs a = rowsf_args(p, ps, pb, act, nullptr, q);
#ifdef PO2Q_ROWS_DIAG
    if (const char* dv = getenv("PO2Q_ROWSF_DEBUG")) {
        const int dbg = atoi(dv);
#define PO2Q_RFD(v)                                                                                             \
    if (dbg == v && p.C == 16 && p.pd == 4 && p.nts == 1 && p.PS == 1 && !epi)                                 \
        return launch_rowsf_t<16, 4, false, 1, 1, false, v>(p, a, x, packed, scale, bias, y, s);             \
    if (dbg == v && p.C == 32 && p.pd == 2 && p.nts == 0 && p.PS == 0 && !epi)                                 \
        return launch_rowsf_t<32, 2, false, 0, 0, false, v>(p, a, x, packed, scale, bias, y, s);
        PO2Q_RFD(1) PO2Q_RFD(2) PO2Q_RFD(3) PO2Q_RFD(4) PO2Q_RFD(8) PO2Q_RFD(5) PO2Q_RFD(10) PO2Q_RFD(11)
#undef PO2Q_RFD
    }
#endif
#define PO2Q_RF(c, d, e, nt, v)                                        \
    if (p.C == c && p.pd == d && epi == e && p.nts == nt && p.PS == v) \
        return launch_rowsf_t<c, d, e, nt, v>(p, a, x, packed, scale, bias, y, s);
#define PO2Q_RF16(d, e) \
    PO2Q_RF(16, d, e, 0, 0) PO2Q_RF(16, d, e, 1, 0) PO2Q_RF(16, d, e, 0, 1) PO2Q_RF(16, d, e, 1, 1) PO2Q_RF(16, d, e, 0, 2) \
    PO2Q_RF(16, d, e, 3, 0) PO2Q_RF(16, d, e, 3, 1)
    PO2Q_RF16(3, false) PO2Q_RF16(4, false) PO2Q_RF16(3, true) PO2Q_RF16(4, true)
    PO2Q_RF(32, 2, false, 0, 0) PO2Q_RF(32, 3, false, 0, 0) PO2Q_RF(32, 4, false, 0, 0)
    PO2Q_RF(32, 2, true, 0, 0) PO2Q_RF(32, 3, true, 0, 0) PO2Q_RF(32, 4, true, 0, 0)
    PO2Q_RF(32, 2, false, 0, 1) PO2Q_RF(32, 3, false, 0, 1) PO2Q_RF(32, 4, false, 0, 1)
    PO2Q_RF(32, 2, true, 0, 1) PO2Q_RF(32, 3, true, 0, 1) PO2Q_RF(32, 4, true, 0, 1)
    PO2Q_RF(32, 2, false, 2, 0) PO2Q_RF(32, 3, false, 2, 0) PO2Q_RF(32, 4, false, 2, 0)
    PO2Q_RF(32, 2, true, 2, 0) PO2Q_RF(32, 3, true, 2, 0) PO2Q_RF(32, 4, true, 2, 0)
    PO2Q_RF(32, 2, false, 2, 1) PO2Q_RF(32, 3, false, 2, 1) PO2Q_RF(32, 4, false, 2, 1)
    PO2Q_RF(32, 2, true, 2, 1) PO2Q_RF(32, 3, true, 2, 1) PO2Q_RF(32, 4, true, 2, 1)
#undef PO2Q_RF16
#undef PO2Q_RF
    return hipErrorInvalidValue;
}

// The residual add inside the kernel: every full-row plan whose residual ring fits in LDS.
bool rowsf_res_ok(const ConvPlan& p) { return rowsf_plan_ok(p) && rowsf_res_lds(p) <= 160 * 1024; }

hipError_t launch_conv_rowsf_res(const ConvPlan& p, const float* x, const uint16_t* packed, const float* scale,
                                 const float* bias, float* y, const float* ps, const float* pb, const float* res,
                                 int act, hipStream_t s, const WQuant& q) {
    if (!rowsf_res_ok(p) || !res) return hipErrorInvalidValue;
    const RowsFArgs a = rowsf_args(p, ps, pb, act, res, q);
#define PO2Q_RFR(c, d, nt, v)                            \
    if (p.C == c && p.pd == d && p.nts == nt && p.PS == v) \
        return launch_rowsf_t<c, d, true, nt, v, true>(p, a, x, packed, scale, bias, y, s);
    PO2Q_RFR(16, 3, 0, 0) PO2Q_RFR(16, 3, 1, 0) PO2Q_RFR(16, 3, 0, 1) PO2Q_RFR(16, 3, 1, 1) PO2Q_RFR(16, 3, 0, 2)
    PO2Q_RFR(16, 4, 0, 0) PO2Q_RFR(16, 4, 1, 0) PO2Q_RFR(16, 4, 0, 1) PO2Q_RFR(16, 4, 1, 1) PO2Q_RFR(16, 4, 0, 2)
    PO2Q_RFR(32, 2, 0, 0) PO2Q_RFR(32, 3, 0, 0) PO2Q_RFR(32, 4, 0, 0)
    PO2Q_RFR(32, 2, 0, 1) PO2Q_RFR(32, 3, 0, 1) PO2Q_RFR(32, 4, 0, 1)
    PO2Q_RFR(16, 3, 3, 0) PO2Q_RFR(16, 3, 3, 1) PO2Q_RFR(16, 4, 3, 0) PO2Q_RFR(16, 4, 3, 1)
    PO2Q_RFR(32, 2, 2, 0) PO2Q_RFR(32, 3, 2, 0) PO2Q_RFR(32, 4, 2, 0)
    PO2Q_RFR(32, 2, 2, 1) PO2Q_RFR(32, 3, 2, 1) PO2Q_RFR(32, 4, 2, 1)
#undef PO2Q_RFR
    return hipErrorInvalidValue;
}

}  // namespace po2q
