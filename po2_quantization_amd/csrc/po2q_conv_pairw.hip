// The stage-2 conv pair (C = 32 -> 32 -> 32, 3x3 / stride 1 / pad 1, W <= 128) as FOUR waves of 32
// output columns -- one wave per SIMD, every weight fragment of both convs in registers:
//   y = act2(Q(w2) * act1(Q(w1) * x [* ps1 + pb1]) [* ps2 + pb2] (+ res))
// the two QuantizedConv2d of a ResNet56 stage-2 BasicBlock (reference models/resnet.py:55-71; each
// conv is QuantizedConv2d.forward, models/quantized_conv.py:32-38) with the block's eval BatchNorm /
// ReLU between and after them.  Same row walk and arithmetic as conv_pair (po2q_conv_pair.hip: full-row
// block per (image, segment of rows), x rows LDS-DMA'd into a PD-slot raw ring, exact bf16x3 split,
// the intermediate kept split in a 2-slot LDS ring, one s_barrier per step, row reuse over the 3 tap
// rows, hand-counted vmcnt), with the block's work spread differently:
//   conv_pair<32>: 7 waves x 16 columns, 2 waves on three SIMDs and 1 on the fourth, 210 VGPRs each
//     (512-register file / 2 waves), so conv 2's 18 B fragments live in LDS: every conv-2 MFMA
//     group waits on an LDS read of its weights (the stamps' conv-2 phase is twice conv 1's);
//   conv_pairw: 4 waves x 32 columns (2 pixel groups), one per SIMD, up to 512 registers each: both
//     convs' 36 B fragments stay in VGPRs, every A fragment read feeds 6 MFMAs (3 tap rows x 2
//     tiles), and a wave's stores cover whole 128-byte lines (its 32 columns of a channel: one
//     row_ror:8 DPP exchange per value, as the C = 16 pair does), where 16-column waves stored half
//     lines (1.34x the output bytes in write traffic, profiles/r05_pmc_pair32.json).
// At W = 112 the fourth wave's second group (columns 112-127) is image padding: its MFMAs run on
// zeros and its stores are dropped, so every SIMD carries the same 2 groups (the 7-strip block put 2
// strips on three SIMDs and 1 on the fourth: the same busiest-SIMD load, 2 x 16 columns).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdint>
#include <cstdlib>
#include <string>
#include <type_traits>
#include <utility>

#include "../../include/po2q.h"
#include "po2q_epi.h"
#include "po2q_internal.h"
#include "po2q_quant_dev.h"
#include "po2q_rows_dev.h"
#include "po2q_x3_dev.h"

#ifndef PO2Q_PAIRW_VA
#define PO2Q_PAIRW_VA 1  // vector instructions per MFMA issue gap in phase A (x split beside conv 2)
#endif
#ifndef PO2Q_PAIRW_VB
#define PO2Q_PAIRW_VB 2  // ... in phase B (both epilogues beside conv 1)
#endif

namespace po2q {

namespace {
constexpr int kPWC = 32;                           // channels (C = K)
constexpr int kPWSW = 32;                          // output columns per wave
constexpr int kPWWaves = 4;
constexpr int kPWWp = kPWSW * kPWWaves;            // padded row width (128 columns)
constexpr int kPWPL = (kPWSW + 2) * 2 * kPWC + 32;  // a wave's x plane: [34 px][32 ch] bf16 (+ pad)
constexpr int kPWYPL = (kPWWp + 3) * 2 * kPWC;      // a shared intermediate plane: [131 px][32 ch] bf16
constexpr int kPWRes = kPWSW * kPWC * 4;            // a wave's residual slot: [32 ch][32 px] fp32
constexpr int kPWRaw = kPWC * kPWWp * 4;            // a raw x slot: [32 ch][128 px] fp32
constexpr int kPWRPB = kPWWp * 4;                   // raw row pitch (bytes per channel row)

// byte offset of channel octet oc of pixel P in a [pixel][32 ch] bf16 plane, octets XOR-swizzled by
// (P >> 1) & 3 (x_addr<32> of po2q_x3_dev.h; conv_pair's yoct<32>)
__device__ __forceinline__ int pw_oct(int P, int oc) { return P * 64 + 16 * (oc ^ ((P >> 1) & 3)); }

// f(integral_constant<int, 0>), ..., f(integral_constant<int, N - 1>) in order
template <class F, int... R>
__device__ __forceinline__ void pw_unroll(F& f, std::integer_sequence<int, R...>) {
    (f(std::integral_constant<int, R>{}), ...);
}
}  // namespace

struct PairWArgs {
    int N, H, W;
    int RB, nseg, items, remap;
    WQuant q1, q2;
    const float* b1;  // conv biases (NULL: none)
    const float* b2;
    const float* ps1;  // epilogue 1 / 2: v * ps[k] + pb[k], then the activation (NULL parts skipped)
    const float* pb1;
    const float* ps2;
    const float* pb2;
    int act1, act2;
    const float* res;  // RES: residual [N, C, H, W] added before act2
};

// PD: x ring slots (2 or 3); NTS bit 0: non-temporal stores, bit 1: non-temporal x loads.
// E: 0 = plain chain (y = scale * acc), 1 = general epilogues, 2 = the BasicBlock form (ReLU after both
// BNs, the conv scale and bias folded into the BN affine at staging).
template <int PD, int NTS, bool RES, int E>
__global__ __launch_bounds__(256, 1) void conv_pairw(const float* __restrict__ x, float* __restrict__ y,
                                                     PairWArgs a) {
    static_assert(PD == 2 || PD == 3, "raw ring slots");
    constexpr int CC = kPWC, SW = kPWSW, WC = SW + 2, PL = kPWPL, YPL = kPWYPL, RPB = kPWRPB;
    constexpr int NG = SW / 16, NT = CC / 16, KS = 3, NF = 3 * KS * NT;
    constexpr int yslot = 3 * YPL;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    unsigned char* raw = lds;                                             // PD x [32][128] fp32
    unsigned char* yr = raw + PD * kPWRaw;                                // 2 x 3 planes (intermediate)
    unsigned char* slab = yr + 2 * yslot + wave * (3 * PL);               // this wave's x planes
    unsigned char* resr = yr + 2 * yslot + kPWWaves * 3 * PL + wave * (PD * kPWRes);

    int blk = blockIdx.x;
    if (a.remap) blk = (blk & 7) * (int)(gridDim.x >> 3) + (blk >> 3);
    if (blk >= a.items) return;  // block-uniform
    const int seg = blk % a.nseg;
    const int n = blk / a.nseg;
    const int p0 = seg * a.RB;
    const int rbe = min(a.RB, a.H - p0);
    const int nx = rbe + 4;     // x rows p0-2 .. p0+rbe+1
    const int n1 = rbe + 2;     // intermediate rows p0-1 .. p0+rbe
    // the conv-1 epilogue of a step runs in the NEXT step (beside its MFMAs), so conv 2 takes
    // intermediate row j - 4 at step j and output row p0 + o completes at step o + 6
    const int nsteps = nx + 2;
    const int q0 = wave * SW;
    const int HW = a.H * a.W;

    // ---- x DMA: instruction i of wave w, lane l -> float4 e = 64 (4 w + i) + l of the row's
    // [32][128 / 4] float4 (columns >= W load out of range: zeros)
    const __amdgpu_buffer_rsrc_t rs = rows_rsrc(x + (int64_t)n * CC * HW, CC * HW * 4);
    uint32_t vi[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int e = 64 * (4 * wave + i) + lane;
        const int c = e >> 5, q = 4 * (e & 31);
        vi[i] = q < a.W ? ((uint32_t)c * (uint32_t)HW + (uint32_t)q) * 4u : 0x7fffffffu;
    }
    const uint32_t raw_lds = (uint32_t)(uintptr_t)raw;
    // residual of this wave's strip: [32 ch][32 px], instruction i, lane l -> float4 64 i + l
    const __amdgpu_buffer_rsrc_t rres = rows_rsrc(RES ? a.res + (int64_t)n * CC * HW : x, RES ? CC * HW * 4 : 4);
    uint32_t vr[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int e = 64 * i + lane;
        const int c = e >> 3, q = q0 + 4 * (e & 7);
        vr[i] = q < a.W ? ((uint32_t)c * (uint32_t)HW + (uint32_t)q) * 4u : 0x7fffffffu;
    }
    const uint32_t res_lds = (uint32_t)(uintptr_t)resr;
    // x row jn into raw slot sl; with RES the residual of the output row stored at step jn
    auto load_row = [&](int sl, int jn) __attribute__((always_inline)) {
        const int h = p0 - 2 + jn;
        const bool hok = jn < nx && h >= 0 && h < a.H;
        const uint32_t roff = (uint32_t)(hok ? h : 0) * (uint32_t)a.W * 4u;
        const uint32_t base = raw_lds + (uint32_t)(sl * kPWRaw) + (uint32_t)(4 * wave) * 1024u;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            rows_dma16<(NTS & 2) != 0>(rs, (hok && vi[i] != 0x7fffffffu) ? vi[i] + roff : 0x7fffffffu, 0u,
                                       base + i * 1024u);
        if constexpr (RES) {
            const int o = jn - 6;
            const bool ook = jn >= 6 && o < rbe;
            const uint32_t ooff = (uint32_t)(ook ? p0 + o : 0) * (uint32_t)a.W * 4u;
#pragma unroll
            for (int i = 0; i < 4; ++i)
                rows_dma16<false>(rres, (ook && vr[i] != 0x7fffffffu) ? vr[i] + ooff : 0x7fffffffu, 0u,
                                  res_lds + (uint32_t)(sl * kPWRes) + i * 1024u);
        }
    };

    // ---- x split: lane -> columns 2 cp, 2 cp + 1 of the strip (cp = lane & 15), channel octet so =
    // lane >> 4; one ds_read_b64 per channel reads both columns.  Halo lanes: lane -> (side, channel)
    // of the neighbours' columns in the shared raw row (zero outside the image)
    const int cp = lane & 15, so = lane >> 4;
    const int rdx0 = (so * 8) * RPB + (q0 + 2 * cp) * 4;
    const int wa0 = pw_oct(2 * cp + 1, so), wa1 = pw_oct(2 * cp + 2, so);
    const int hl = lane & 31;
    const int hside = hl >> 4, hch = 16 * (lane >> 5) + (hl & 15);
    const int hq = hside ? q0 + SW : q0 - 1;
    const bool h_ok = hq >= 0 && hq < a.W;
    const int wa_h = pw_oct(hside ? WC - 1 : 0, hch >> 3) + (hch & 7) * 2;
    const int rdx_h = hch * RPB + (h_ok ? hq : 0) * 4;
    // A / B fragment addresses (one b128 each): x planes (pixel = strip column + 1 - 1 + tap) and the
    // shared intermediate planes (pixel = column + 1 - 1 + tap), k = octet g of the tap's 32 channels
    int aoff[NG][KS], yoff[NG][KS];
    {
        const int p = lane & 15, g = lane >> 4;
#pragma unroll
        for (int grp = 0; grp < NG; ++grp)
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                aoff[grp][ks] = pw_oct(16 * grp + p + ks, g);
                yoff[grp][ks] = pw_oct(q0 + 16 * grp + p + ks, g);
            }
    }

    const __amdgpu_buffer_rsrc_t ry = rows_rsrc(y + (int64_t)n * CC * HW, CC * HW * 4);
    constexpr int ST = 2 * NT;             // stores per step (whole-line pairs; dropped ones out of range)
    constexpr int LD = RES ? 8 : 4;        // DMAs per step
    constexpr int VMW = ST + (PD - 2) * (LD + ST);

    float scale1 = 1.0f, scale2 = 1.0f;
    bool fin1 = true, fin2 = true;
    bf16x8 bw1[NF], bw2[NF];
    float bk1[E ? NT * 4 : 1], e1s[E ? NT * 4 : 1], e1b[E ? NT * 4 : 1];  // conv 1: ch 16 nt + 4 (lane >> 4) + e
    float bk2[NT], e2s[NT], e2b[NT];                                       // conv 2: ch 16 nt + (lane & 15)
    floatx4 acc1[3][NG][NT], acc2[3][NG][NT];
#pragma unroll
    for (int sl = 0; sl < 3; ++sl)
#pragma unroll
        for (int grp = 0; grp < NG; ++grp)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
                acc1[sl][grp][nt] = floatx4{0.f, 0.f, 0.f, 0.f};
                acc2[sl][grp][nt] = floatx4{0.f, 0.f, 0.f, 0.f};
            }

    // ---- the MFMAs of one split row with vector work threaded between them.  3 tap rows x 3 k-steps x
    // 3 planes x NG groups x NT tiles = 108 MFMAs into the accumulator slots of step S.  TR (conv 1):
    // transposed (A = weights, B = x) on the wave's x planes; else (conv 2): A = the shared intermediate
    // planes, B = weights.  Every A fragment feeds 6 MFMAs (3 tap rows x 2 tiles), which form one region;
    // the 36 MFMAs of a k-step are 6 such regions, and after region
    // r the phase's filler fill(r) issues its piece of vector work: each region is closed by a
    // sched_barrier, so the compiler cannot gather the MFMAs into one run and the vector work into another
    // (with one wave per SIMD no partner wave would fill the matrix pipe during such a vector-only run).
    // Per accumulator the order is k-step major, plane minor, as in conv_pair: the same sums bit for bit.
    auto mfmas = [&](auto S_, auto TR_, floatx4 (&acc)[3][NG][NT], const bf16x8 (&bw)[NF], const unsigned char* pb,
                     auto&& fill) __attribute__((always_inline)) {
        constexpr int SR = decltype(S_)::value;
        constexpr bool TR = decltype(TR_)::value;
        constexpr int SL[3] = {(SR + 1) % 3, SR, (SR + 2) % 3};
        // one register set: fragment (pl, grp) of k-step ks + 1 is read right after its 6 MFMAs of k-step
        // ks (tap rows x tiles), 36 MFMAs ahead of its use
        bf16x8 af[3][NG];
        auto load1 = [&](int ks, int pl, int grp) __attribute__((always_inline)) {
            const int off = TR ? pl * PL + aoff[grp][ks] : pl * YPL + yoff[grp][ks];
            af[pl][grp] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(pb + off));
        };
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
#pragma unroll
            for (int grp = 0; grp < NG; ++grp) load1(0, pl, grp);
        auto region = [&](auto R_) __attribute__((always_inline)) {
            constexpr int R = decltype(R_)::value;
            constexpr int ks = R / 6;
            constexpr int fi = R % 6;                 // fragment (pl, grp) of this region
            constexpr int pl = fi / NG, grp = fi % NG;
#pragma unroll
            for (int m = 0; m < 6; ++m) {             // (r3, nt): tap row 2 first
                const int r3 = m / NT, nt = m % NT;
                const int rr = 2 - r3;
                const bf16x8 b = bw[(rr * KS + ks) * NT + nt];
                // slot SL[0] starts at this step: its first MFMA takes a zero accumulator
                const floatx4 c = (rr == 0 && ks == 0 && pl == 0) ? floatx4{0.f, 0.f, 0.f, 0.f} : acc[SL[rr]][grp][nt];
                acc[SL[rr]][grp][nt] = TR ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, af[pl][grp], c, 0, 0, 0)
                                          : __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[pl][grp], b, c, 0, 0, 0);
            }
            if constexpr (ks + 1 < KS) load1(ks + 1, pl, grp);
            fill(R_);
            __builtin_amdgcn_sched_barrier(0);
        };
        pw_unroll(region, std::make_integer_sequence<int, 18>{});
    };

    // conv 1's completed accumulator slot, moved to VGPRs at the end of a step for the next step's epilogue
    floatx4 pend1[NG][NT];
#pragma unroll
    for (int grp = 0; grp < NG; ++grp)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) pend1[grp][nt] = floatx4{0.f, 0.f, 0.f, 0.f};

    // Step j (one barrier): x row j lands; phase A: conv 2 on intermediate row j - 4 with the exact split of
    // x row j threaded between its MFMAs; phase B: conv 1 on x row j with conv 2's epilogue + stores (output
    // row j - 6, accumulator slot D of phase A) and the deferred conv-1 epilogue (intermediate row j - 3,
    // completed at step j - 1 and held in pend1) threaded between its MFMAs.  No vector task depends on
    // the MFMAs of its own phase.
    auto step = [&](auto S_, int j) __attribute__((always_inline)) {
        constexpr int S6 = decltype(S_)::value;
        constexpr int S = S6 % 3;
        constexpr int D = (S + 2) % 3;          // the accumulator slot that completes
        constexpr int YW = (S6 + 1) & 1;        // ring slot written: intermediate row j - 3
        constexpr int YR = S6 & 1;              // ring slot read: intermediate row j - 4
        const int RS = (6 % PD == 0) ? S6 % PD : j % PD;
        rows_wait<VMW>();  // this wave's part of x row j (and its residual) has landed
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // + everyone's plane writes
        load_row((6 % PD == 0) ? (S6 + PD - 1) % PD : (j - 1 + PD) % PD, j - 1 + PD);
        uint32_t bx[2][8], hx;
        {
            const unsigned char* rw = raw + RS * kPWRaw;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const uint2 v2 = *reinterpret_cast<const uint2*>(rw + rdx0 + e * RPB);
                bx[0][e] = v2.x;
                bx[1][e] = v2.y;
            }
            hx = *reinterpret_cast<const uint32_t*>(rw + rdx_h);
        }
        // ---- phase A filler: the exact split of x row j into this wave's planes (split3 per value:
        // hi = x & 0xffff0000, r1 = x' - hi with x' clamped to +-FLT_MAX, mid = r1 & 0xffff0000, lo = r1 - mid)
        uint32_t mb[2][8], lb[2][8];
        auto fill_a = [&](auto R_) __attribute__((always_inline)) {
            constexpr int R = decltype(R_)::value;
            if constexpr (R < 10 && R % 5 != 4) {  // column c = R / 5, values 2 (R % 5), + 1
                constexpr int c = R / 5;
#pragma unroll
                for (int v = 2 * (R % 5); v < 2 * (R % 5) + 2; ++v) {
                    const float xc = __builtin_amdgcn_fmed3f(__uint_as_float(bx[c][v]), -3.40282347e38f, 3.40282347e38f);
                    const float r1 = xc - __uint_as_float(__float_as_uint(xc) & 0xffff0000u);
                    mb[c][v] = __float_as_uint(r1) & 0xffff0000u;
                    lb[c][v] = __float_as_uint(r1 - __uint_as_float(mb[c][v]));
                }
            } else if constexpr (R < 10) {  // column c: pack the three planes, 3 ds_write_b128
                constexpr int c = R / 5;
                const uint32_t(&b)[8] = bx[c];
                const uint4 hi = make_uint4(pk_hi16(b[0], b[1]), pk_hi16(b[2], b[3]), pk_hi16(b[4], b[5]), pk_hi16(b[6], b[7]));
                const uint4 mid = make_uint4(pk_hi16(mb[c][0], mb[c][1]), pk_hi16(mb[c][2], mb[c][3]),
                                             pk_hi16(mb[c][4], mb[c][5]), pk_hi16(mb[c][6], mb[c][7]));
                const uint4 lo = make_uint4(pk_hi16(lb[c][0], lb[c][1]), pk_hi16(lb[c][2], lb[c][3]),
                                            pk_hi16(lb[c][4], lb[c][5]), pk_hi16(lb[c][6], lb[c][7]));
                const int wa = c ? wa1 : wa0;
                *reinterpret_cast<uint4*>(slab + wa) = hi;
                *reinterpret_cast<uint4*>(slab + PL + wa) = mid;
                *reinterpret_cast<uint4*>(slab + 2 * PL + wa) = lo;
            } else if constexpr (R == 10) {  // the halo lane's value
                uint16_t h16, m16, l16;
                split1(h_ok ? hx : 0u, h16, m16, l16);
                *reinterpret_cast<uint16_t*>(slab + wa_h) = h16;
                *reinterpret_cast<uint16_t*>(slab + PL + wa_h) = m16;
                *reinterpret_cast<uint16_t*>(slab + 2 * PL + wa_h) = l16;
            }
        };
        // ---- phase A: conv 2 on intermediate row j - 4 (unconditional: in the first steps it reads the
        // zeroed ring slots and its outputs are dropped)
        mfmas(std::integral_constant<int, S>{}, std::false_type{}, acc2, bw2, yr + YR * yslot, fill_a);

        // ---- phase B fillers.  Conv 2's epilogue of slot D: lane L holds pixels 4g .. 4g + 3 of each group
        // for channel 16 nt + (L & 15); one row_ror:8 DPP move per value gives store A channels 0-7 and
        // store B channels 8-15 of the tile as whole 128-byte lines.  Then conv 1's deferred epilogue:
        // affine / activation, zeros outside the image (conv 2's padding; a select, not a branch), the
        // exact split and 8 bytes per plane into the shared intermediate ring slot YW.
        const int o = j - 6;
        const bool orow = o >= 0 && o < rbe;
        const unsigned char* rres_row = resr + RS * kPWRes;  // loaded with x row j
        const int g = lane >> 4, p = lane & 15;
        const int qs = q0 + ((lane & 8) ? 16 : 0) + 4 * g;
        const uint32_t rowoff = (uint32_t)(orow ? p0 + o : 0) * a.W + (uint32_t)qs;
        const bool ok = orow && qs < a.W;
        const int i1 = j - 3;  // intermediate row of the deferred epilogue
        const int r1 = p0 - 1 + i1;
        const bool irow = i1 >= 0 && i1 < n1 && r1 >= 0 && r1 < a.H;
        unsigned char* yw = yr + YW * yslot;
        uint32_t eb[NG][NT][4];
        auto fill_b = [&](auto R_) __attribute__((always_inline)) {
            constexpr int R = decltype(R_)::value;
            if constexpr (R < 2) {  // conv 2's epilogue, tile nt = R: values, whole-line exchange, 2 stores
                constexpr int nt = R;
                const int ch = 16 * nt + (lane & 15);
                floatx4 vv[NG];
#pragma unroll
                for (int grp = 0; grp < NG; ++grp) {
                    floatx4 v;
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        v[e] = E == 0 ? acc2[D][grp][nt][e] * scale2 + 0.0f
                               : E == 2 ? acc2[D][grp][nt][e] * e2s[nt] + e2b[nt]  // folded: scale2 * ps2, b2 * ps2 + pb2
                                        : (acc2[D][grp][nt][e] * scale2 + bk2[nt]) * e2s[nt] + e2b[nt];
                    if constexpr (RES) {
                        const floatx4 r = *reinterpret_cast<const floatx4*>(rres_row + ch * (SW * 4) + (16 * grp + 4 * g) * 4);
#pragma unroll
                        for (int e = 0; e < 4; ++e) v[e] += r[e];
                    }
                    if constexpr (E == 2) {
#pragma unroll
                        for (int e = 0; e < 4; ++e) v[e] = v[e] < 0.0f ? 0.0f : v[e];  // ReLU (NaN propagates)
                    } else if constexpr (E != 0) {
#pragma unroll
                        for (int e = 0; e < 4; ++e) v[e] = epi_act(v[e], a.act2);
                    }
                    vv[grp] = v;
                }
                floatx4 sa, sb;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    sa[e] = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(vv[0][e]), __float_as_int(vv[1][e]),
                                                                       0x128, 0xf, 0xc, false));
                    sb[e] = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(vv[1][e]), __float_as_int(vv[0][e]),
                                                                       0x128, 0xf, 0x3, false));
                }
                const uint32_t ca = (uint32_t)(16 * nt) + (uint32_t)(lane & 7), cb = ca + 8u;
                rows_store<(NTS & 1) != 0>(ry, ok ? (ca * (uint32_t)HW + rowoff) * 4u : 0x7fffffffu, sa);
                rows_store<(NTS & 1) != 0>(ry, ok ? (cb * (uint32_t)HW + rowoff) * 4u : 0x7fffffffu, sb);
            } else if constexpr (R >= 2 && R < 10) {  // deferred epilogue 1, quad (grp, nt) = (R - 2) / 2
                constexpr int qd = (R - 2) / 2, grp = qd / NT, nt = qd % NT;
                const int q = q0 + 16 * grp + p;  // lane: pixel q, channels 16 nt + 4 g .. + 3
                if constexpr (R % 2 == 0) {
                    const bool okq = irow && q < a.W;
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        float t;
                        if constexpr (E == 0) {
                            t = pend1[grp][nt][e] * scale1 + 0.0f;
                        } else if constexpr (E == 2) {
                            const int c = nt * 4 + e;
                            t = pend1[grp][nt][e] * e1s[c] + e1b[c];  // folded affine, then ReLU
                            t = t < 0.0f ? 0.0f : t;
                        } else {
                            const int c = nt * 4 + e;
                            t = epi_act((pend1[grp][nt][e] * scale1 + bk1[c]) * e1s[c] + e1b[c], a.act1);
                        }
                        eb[grp][nt][e] = okq ? __float_as_uint(t) : 0u;
                    }
                } else {
                    uint2 h2, m2, l2;
                    split4p<false>(eb[grp][nt], h2, m2, l2);
                    const int wo = pw_oct(q + 1, (4 * nt + g) >> 1) + 8 * (g & 1);
                    *reinterpret_cast<uint2*>(yw + wo) = h2;
                    *reinterpret_cast<uint2*>(yw + YPL + wo) = m2;
                    *reinterpret_cast<uint2*>(yw + 2 * YPL + wo) = l2;
                }
            } else if constexpr (R == 17) {  // conv 1's slot D (complete since k-step 2's first MFMAs)
#pragma unroll
                for (int grp = 0; grp < NG; ++grp)
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt) pend1[grp][nt] = acc1[D][grp][nt];
            }
        };
        // ---- phase B: conv 1 on x row j (transposed MFMAs)
        mfmas(std::integral_constant<int, S>{}, std::true_type{}, acc1, bw1, slab, fill_b);
    };

    // x rows 0 .. PD-2, each followed by ST dropped stores (the steady-state count)
    {
        const floatx4 z = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int r = 0; r < PD - 1; ++r) {
            load_row(r, r);
#pragma unroll
            for (int i = 0; i < ST; ++i) rows_store<(NTS & 1) != 0>(ry, 0x7fffffffu, z);
        }
    }
    // ---- both weights quantized + packed into VGPRs while those DMAs fly (scratch: the intermediate
    // planes, zeroed right after)
    {
        unsigned* red = reinterpret_cast<unsigned*>(yr);
        unsigned* thr = red + 16;
        scale1 = wq_prologue(a.q1, thr, red, kPWWaves, fin1);
#pragma unroll
        for (int f = 0; f < NF; ++f)
            bw1[f] = __builtin_bit_cast(bf16x8, wq_frag_rows(a.q1, CC, CC, CC, NT, KS, f * 64 + lane, scale1, fin1, thr));
        __syncthreads();  // red / thr reads of conv 1 done
        scale2 = wq_prologue(a.q2, thr, red, kPWWaves, fin2);
#pragma unroll
        for (int f = 0; f < NF; ++f)
            bw2[f] = __builtin_bit_cast(bf16x8, wq_frag_rows(a.q2, CC, CC, CC, NT, KS, f * 64 + lane, scale2, fin2, thr));
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
            if constexpr (E != 0) {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int k1 = 16 * nt + 4 * (lane >> 4) + e;
                    bk1[nt * 4 + e] = a.b1 ? a.b1[k1] : 0.0f;
                    e1s[nt * 4 + e] = a.ps1 ? a.ps1[k1] : 1.0f;
                    e1b[nt * 4 + e] = a.pb1 ? a.pb1[k1] : 0.0f;
                }
            }
            const int k2 = 16 * nt + (lane & 15);
            bk2[nt] = (E && a.b2) ? a.b2[k2] : 0.0f;
            e2s[nt] = (E && a.ps2) ? a.ps2[k2] : 1.0f;
            e2b[nt] = (E && a.pb2) ? a.pb2[k2] : 0.0f;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every staged value lands here
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
            if constexpr (E != 0) {
#pragma unroll
                for (int e = 0; e < 4; ++e) asm volatile("" : "+v"(bk1[nt * 4 + e]), "+v"(e1s[nt * 4 + e]), "+v"(e1b[nt * 4 + e]));
            }
            asm volatile("" : "+v"(bk2[nt]), "+v"(e2s[nt]), "+v"(e2b[nt]));
        }
#pragma unroll
        for (int f = 0; f < NF; ++f) asm volatile("" : "+v"(bw1[f]), "+v"(bw2[f]));
        if constexpr (E == 2) {  // BasicBlock form: the conv scale and bias folded into the affine
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int c = nt * 4 + e;
                    e1b[c] = bk1[c] * e1s[c] + e1b[c];
                    e1s[c] = scale1 * e1s[c];
                }
                e2b[nt] = bk2[nt] * e2s[nt] + e2b[nt];
                e2s[nt] = scale2 * e2s[nt];
            }
        }
        __syncthreads();  // scratch reads done: zero the intermediate planes (padding columns)
        for (int e = tid; e < (2 * yslot) / 16; e += blockDim.x)
            reinterpret_cast<uint4*>(yr)[e] = make_uint4(0u, 0u, 0u, 0u);
        // step 0's barrier publishes the zeros
    }
    for (int j = 0; j < nsteps; j += 6) {
        step(std::integral_constant<int, 0>{}, j);
        step(std::integral_constant<int, 1>{}, j + 1);
        step(std::integral_constant<int, 2>{}, j + 2);
        if (j + 3 >= nsteps) break;
        step(std::integral_constant<int, 3>{}, j + 3);
        step(std::integral_constant<int, 4>{}, j + 4);
        step(std::integral_constant<int, 5>{}, j + 5);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // trailing DMAs land before the wave ends
}

namespace {

size_t pairw_lds(int pd, bool res) {
    return (size_t)pd * kPWRaw + 2 * 3 * (size_t)kPWYPL + (size_t)kPWWaves * 3 * kPWPL +
           (res ? (size_t)kPWWaves * pd * kPWRes : 0);
}

template <int PD, int NTS>
hipError_t launch_pairw_t(int blocks, size_t lds, const PairWArgs& a, const float* x, float* y, bool res, hipStream_t s) {
    const bool plain = !res && !a.b1 && !a.b2 && !a.ps1 && !a.pb1 && !a.ps2 && !a.pb2 && a.act1 == 0 && a.act2 == 0;
    const dim3 grid((unsigned)blocks), block(64 * kPWWaves);
    if (plain) {
        hipLaunchKernelGGL((conv_pairw<PD, NTS, false, 0>), grid, block, lds, s, x, y, a);
        return hipGetLastError();
    }
    if constexpr (PD == 2) {  // the residual slots leave room for 2 x slots only
        if (res && a.act1 == 1 && a.act2 == 1)  // the BasicBlock form (resnet.py:55-71): ReLU / ReLU
            hipLaunchKernelGGL((conv_pairw<PD, NTS, true, 2>), grid, block, lds, s, x, y, a);
        else if (res)
            hipLaunchKernelGGL((conv_pairw<PD, NTS, true, 1>), grid, block, lds, s, x, y, a);
        else
            hipLaunchKernelGGL((conv_pairw<PD, NTS, false, 1>), grid, block, lds, s, x, y, a);
        return hipGetLastError();
    }
    return hipErrorInvalidValue;
}

// PO2Q_PAIR_W32: 0 turns the 4-wave kernel off (A/B runs: conv_pair<32> takes the shape), a number
// 2 / 3 sets the plain form's ring depth; PO2Q_PAIR_W32_NTS the store / load policy (default 3:
// non-temporal x loads and y stores)
int pairw_knob() {
    const char* e = getenv("PO2Q_PAIR_W32");
    if (!e) return 0;  // measured slower than conv_pair<32> (0.419 vs 0.356 ms, profiles/r06_pairw_ab.jsonl): off
    return atoi(e);
}

}  // namespace

bool pairw_applicable(int64_t N, int64_t C, int64_t H, int64_t W) {
    return C == 32 && W > 3 * kPWSW && W <= kPWWp && W % 4 == 0 && N > 0 && H > 0 && pairw_knob() != 0 &&
           (int64_t)C * H * W * 4 < (1LL << 31);
}

hipError_t pairw_launch(const float* x, const float* w1, const float* w2, float* y, int64_t N, int64_t H,
                        int64_t W, int bits, int fsr, int mode, const float* bias1, const float* bias2,
                        const float* post_scale1, const float* post_shift1, int act1, const float* post_scale2,
                        const float* post_shift2, const float* residual, int act2, hipStream_t s) {
    const bool res = residual != nullptr;
    int pd = pairw_knob();
    const bool plain = !res && !bias1 && !bias2 && !post_scale1 && !post_shift1 && !post_scale2 && !post_shift2 &&
                       act1 == 0 && act2 == 0;
    if (pd != 3 || !plain) pd = 2;  // the residual slots leave room for 2 x slots only
    // non-temporal x loads and y stores, except with a residual: the residual re-reads x a few steps
    // after its row's DMA, which temporal loads leave in L2 (conv_pair's variant 21 at C = 16)
    int nts = res ? 1 : 3;
    if (const char* e = getenv("PO2Q_PAIR_W32_NTS")) nts = atoi(e) == 1 ? 1 : 3;
    const size_t lds = pairw_lds(pd, res);
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    int nseg = std::max<int64_t>(1, (256 + N - 1) / N);
    nseg = std::min<int>(nseg, std::max<int>(1, (int)H / 8));
    PairWArgs a;
    a.N = (int)N; a.H = (int)H; a.W = (int)W;
    a.RB = (int)((H + nseg - 1) / nseg);
    a.nseg = (int)((H + a.RB - 1) / a.RB);
    const int64_t items = N * a.nseg;
    if (items > INT_MAX / 2) return hipErrorInvalidValue;
    const int blocks = (int)((items + 7) / 8 * 8);
    a.items = (int)items;
    a.remap = (blocks % 8 == 0) ? 1 : 0;
    const int lo = fsr - (1 << (bits - 1)), hi = fsr - 1;
    a.q1.w = w1; a.q1.n = 32 * 32 * 9; a.q1.lo = lo; a.q1.hi = hi; a.q1.mode = mode - 1;
    a.q2 = a.q1;
    a.q2.w = w2;
    a.b1 = bias1; a.b2 = bias2;
    a.ps1 = post_scale1; a.pb1 = post_shift1; a.act1 = act1;
    a.ps2 = post_scale2; a.pb2 = post_shift2; a.act2 = act2;
    a.res = residual;
#define PO2Q_PW(d, t) \
    if (pd == d && nts == t) return launch_pairw_t<d, t>(blocks, lds, a, x, y, res, s);
    PO2Q_PW(2, 3)
#ifndef PO2Q_PAIRW_ISA
    PO2Q_PW(3, 3) PO2Q_PW(2, 1)
#endif
#undef PO2Q_PW
    return hipErrorInvalidValue;
}

}  // namespace po2q
