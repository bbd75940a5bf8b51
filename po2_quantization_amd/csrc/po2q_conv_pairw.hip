// The stage-2 conv pair (C = 32 -> 32 -> 32, 3x3 / stride 1 / pad 1, 96 < W <= 128) with the two
// convs given to different waves, every weight fragment in registers:
//   y = act2(Q(w2) * act1(Q(w1) * x [* ps1 + pb1]) [* ps2 + pb2] (+ res))
// the two QuantizedConv2d of a ResNet56 stage-2 BasicBlock (reference models/resnet.py:55-71; each
// conv is QuantizedConv2d.forward, models/quantized_conv.py:32-38) with the block's eval BatchNorm /
// ReLU between and after them.  Same row walk and arithmetic as conv_pair (po2q_conv_pair.hip: full-row
// block per (image, segment of rows), x rows LDS-DMA'd into a PD-slot raw ring, exact bf16x3 split,
// the intermediate kept split in a 2-slot LDS ring, one s_barrier per step, row reuse over the 3 tap
// rows, hand-counted vmcnt), with the block's work spread differently:
//   conv_pair<32>: 7 waves x 16 columns running both convs, 2 waves on three SIMDs and 1 on the
//     fourth, 210 VGPRs each, so conv 2's 18 B fragments live in LDS and every conv-2 MFMA group
//     waits on an LDS read of its weights (the stamps' conv-2 phase is twice conv 1's);
//   conv_pairw: 8 waves on 4 strips of 32 columns.  Waves 0-3 ("B") run conv 1 of strip w: the x DMAs,
//     the exact split, 108 transposed MFMAs per step and (one step later) epilogue 1 into the shared
//     intermediate ring; waves 4-7 ("A") run conv 2 of strip w - 4 on that ring: 108 MFMAs and epilogue 2
//     with its stores.  Each wave holds one conv's 18 B fragments in VGPRs; every A-fragment read feeds 6
//     MFMAs (3 tap rows x 2 tiles); a wave's stores cover its 32 columns of a channel (one row_ror:8 DPP
//     exchange per value, as the C = 16 pair does) where 16-column waves stored half lines.  Wave w and
//     w + 4 share a SIMD, so each SIMD pairs a conv-1 wave with a conv-2 wave: after the barrier A issues
//     MFMAs while B issues its vector work (deferred epilogue 1, split), and B's MFMAs run beside A's
//     epilogue -- the two waves of a SIMD are in opposite phases by construction, where conv_pair's two
//     waves issue their MFMAs, then their vector work, at the same time.
// At W = 112 strip 3's second group (columns 112-127) is image padding: its MFMAs run on zeros and its
// stores are dropped, so every SIMD carries the same 2 groups of both convs.
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
// DBG (diagnostic builds only, -DPO2Q_PAIRW_DIAG, PO2Q_PAIR_W32_DBG; timing only, outputs are wrong):
// bit 1 no MFMAs, 2 no x DMAs, 4 no stores, 8 no epilogue / split vector work, 16 no per-step barrier.
template <int PD, int NTS, bool RES, int E, int DBG = 0>
__global__ __launch_bounds__(512, 1) void conv_pairw(const float* __restrict__ x, float* __restrict__ y,
                                                     PairWArgs a) {
    static_assert(PD >= 2 && PD <= 5, "raw ring slots");
    constexpr int CC = kPWC, SW = kPWSW, WC = SW + 2, PL = kPWPL, YPL = kPWYPL, RPB = kPWRPB;
    constexpr int NG = SW / 16, NT = CC / 16, KS = 3, NF = 3 * KS * NT;
    constexpr int yslot = 3 * YPL;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool roleA = wave >= kPWWaves;  // wave-uniform: conv 2 (A) or conv 1 (B)
    const int sw = wave & (kPWWaves - 1);  // strip
    unsigned char* raw = lds;                                             // PD x [32][128] fp32
    unsigned char* yr = raw + PD * kPWRaw;                                // 2 x 3 planes (intermediate)
    unsigned char* slab = yr + 2 * yslot + sw * (3 * PL);                 // B: this strip's x planes
    unsigned char* resr = yr + 2 * yslot + kPWWaves * 3 * PL + sw * (PD * kPWRes);  // A: residual slots

    int blk = blockIdx.x;
    if (a.remap) blk = (blk & 7) * (int)(gridDim.x >> 3) + (blk >> 3);
    if (blk >= a.items) return;  // block-uniform
    const int seg = blk % a.nseg;
    const int n = blk / a.nseg;
    const int p0 = seg * a.RB;
    const int rbe = min(a.RB, a.H - p0);
    const int nx = rbe + 4;     // x rows p0-2 .. p0+rbe+1
    const int n1 = rbe + 2;     // intermediate rows p0-1 .. p0+rbe
    // epilogue 1 of a step runs at the start of the NEXT step (B's vector phase), so conv 2 takes
    // intermediate row j - 4 at step j and output row p0 + o completes at step o + 6
    const int nsteps = nx + 2;
    const int q0 = sw * SW;
    const int HW = a.H * a.W;

    // ---- B: x DMA, instruction i of strip s, lane l -> float4 e = 64 (4 s + i) + l of the row's
    // [32][128 / 4] float4 (columns >= W load out of range: zeros)
    const __amdgpu_buffer_rsrc_t rs = rows_rsrc(x + (int64_t)n * CC * HW, CC * HW * 4);
    uint32_t vi[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int e = 64 * (4 * sw + i) + lane;
        const int c = e >> 5, q = 4 * (e & 31);
        vi[i] = q < a.W ? ((uint32_t)c * (uint32_t)HW + (uint32_t)q) * 4u : 0x7fffffffu;
    }
    const uint32_t raw_lds = (uint32_t)(uintptr_t)raw;
    auto load_x = [&](int sl, int jn) __attribute__((always_inline)) {
        const int h = p0 - 2 + jn;
        const bool hok = jn < nx && h >= 0 && h < a.H;
        const uint32_t roff = (uint32_t)(hok ? h : 0) * (uint32_t)a.W * 4u;
        const uint32_t base = raw_lds + (uint32_t)(sl * kPWRaw) + (uint32_t)(4 * sw) * 1024u;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            rows_dma16<(NTS & 2) != 0>(rs, (hok && vi[i] != 0x7fffffffu) ? vi[i] + roff : 0x7fffffffu, 0u,
                                       base + i * 1024u);
    };
    // ---- A (RES): the residual of the output row stored at step jn, [32 ch][32 px] of the strip,
    // instruction i, lane l -> float4 64 i + l
    const __amdgpu_buffer_rsrc_t rres = rows_rsrc(RES ? a.res + (int64_t)n * CC * HW : x, RES ? CC * HW * 4 : 4);
    uint32_t vr[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int e = 64 * i + lane;
        const int c = e >> 3, q = q0 + 4 * (e & 7);
        vr[i] = q < a.W ? ((uint32_t)c * (uint32_t)HW + (uint32_t)q) * 4u : 0x7fffffffu;
    }
    const uint32_t res_lds = (uint32_t)(uintptr_t)resr;
    auto load_res = [&](int sl, int jn) __attribute__((always_inline)) {
        const int o = jn - 6;
        const bool ook = jn >= 6 && o < rbe;
        const uint32_t ooff = (uint32_t)(ook ? p0 + o : 0) * (uint32_t)a.W * 4u;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            rows_dma16<false>(rres, (ook && vr[i] != 0x7fffffffu) ? vr[i] + ooff : 0x7fffffffu, 0u,
                              res_lds + (uint32_t)(sl * kPWRes) + i * 1024u);
    };

    // ---- B: x split: lane -> columns 2 cp, 2 cp + 1 of the strip (cp = lane & 15), channel octet so =
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
    // A-fragment addresses (one b128 each): B's x planes (pixel = strip column + tap), A's shared
    // intermediate planes (pixel = column + tap), k = octet g of the tap's 32 channels
    int foff[NG][KS];
    {
        const int p = lane & 15, g = lane >> 4;
#pragma unroll
        for (int grp = 0; grp < NG; ++grp)
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) foff[grp][ks] = pw_oct((roleA ? q0 : 0) + 16 * grp + p + ks, g);
    }

    const __amdgpu_buffer_rsrc_t ry = rows_rsrc(y + (int64_t)n * CC * HW, CC * HW * 4);
    constexpr int ST = 2 * NT;  // A's stores per step (whole-line pairs; dropped ones out of range)
    // counted waits at the top of a step: B waits for its DMAs of x row j (issued PD - 1 steps
    // earlier; its later DMAs may fly), A (RES) for its residual DMAs of the row it stores at step j
    constexpr int VMW_B = 4 * (PD - 2);
    constexpr int VMW_A = ST + (PD - 2) * (4 + ST);

    float scale = 1.0f;  // this wave's conv: scale1 (B) or scale2 (A)
    bool fin = true;
    bf16x8 bw[NF] = {};
    float bk[E ? NT * 4 : 1], es[E ? NT * 4 : 1], eb[E ? NT * 4 : 1];  // B: ch 16 nt + 4 (lane >> 4) + e; A: e = 0
    floatx4 acc[3][NG][NT];
#pragma unroll
    for (int sl = 0; sl < 3; ++sl)
#pragma unroll
        for (int grp = 0; grp < NG; ++grp)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) acc[sl][grp][nt] = floatx4{0.f, 0.f, 0.f, 0.f};

    // The 108 MFMAs of one split row: 3 tap rows x 3 k-steps x 3 planes x NG groups x NT tiles into the
    // accumulator slots of step S.  TR (B, conv 1): transposed (A = weights, B = x) on the strip's x
    // planes; else (A, conv 2): A = the shared intermediate planes, B = weights.  Every fragment feeds 6
    // MFMAs; fragment (pl, grp) of k-step ks + 1 is read right after its 6 MFMAs of k-step ks.  Per
    // accumulator the order is k-step major, plane minor, as in conv_pair: the same sums bit for bit.
    auto mfmas = [&](auto S_, auto TR_, const unsigned char* pb) __attribute__((always_inline)) {
        constexpr int SR = decltype(S_)::value;
        constexpr bool TR = decltype(TR_)::value;
        constexpr int SL[3] = {(SR + 1) % 3, SR, (SR + 2) % 3};
        constexpr int PLS = TR ? PL : YPL;
        bf16x8 af[3][NG];
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
#pragma unroll
            for (int grp = 0; grp < NG; ++grp)
                af[pl][grp] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(pb + pl * PLS + foff[grp][0]));
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
#pragma unroll
            for (int pl = 0; pl < 3; ++pl)
#pragma unroll
                for (int grp = 0; grp < NG; ++grp) {
#pragma unroll
                    for (int m = 0; m < 6; ++m) {  // (r3, nt): tap row 2 first
                        const int r3 = m / NT, nt = m % NT;
                        const int rr = 2 - r3;
                        const bf16x8 b = bw[(rr * KS + ks) * NT + nt];
                        // slot SL[0] starts at this step: its first MFMA takes a zero accumulator
                        const floatx4 c = (rr == 0 && ks == 0 && pl == 0) ? floatx4{0.f, 0.f, 0.f, 0.f}
                                                                         : acc[SL[rr]][grp][nt];
                        acc[SL[rr]][grp][nt] = TR ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, af[pl][grp], c, 0, 0, 0)
                                                  : __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[pl][grp], b, c, 0, 0, 0);
                    }
                    if (ks + 1 < KS)
                        af[pl][grp] = __builtin_bit_cast(
                            bf16x8, *reinterpret_cast<const uint4*>(pb + pl * PLS + foff[grp][ks + 1 < KS ? ks + 1 : 0]));
                }
    };

    // a skipped row's step: only the slot that starts at step S (mfmas' zero accumulator) changes
    auto zero_slot = [&](auto S_) __attribute__((always_inline)) {
        constexpr int SR = decltype(S_)::value;
#pragma unroll
        for (int grp = 0; grp < NG; ++grp)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) acc[(SR + 1) % 3][grp][nt] = floatx4{0.f, 0.f, 0.f, 0.f};
    };

    // B: conv 1's completed accumulator slot, held in VGPRs until the next step's epilogue 1
    floatx4 pend[NG][NT];
#pragma unroll
    for (int grp = 0; grp < NG; ++grp)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) pend[grp][nt] = floatx4{0.f, 0.f, 0.f, 0.f};

    // ---- B, step j: epilogue 1 of intermediate row j - 3 (pend, completed at step j - 1) into ring slot
    // YW, the exact split of x row j, conv 1 on it (intermediate row j - 2 completes into pend)
    auto stepB = [&](auto S_, int j) __attribute__((always_inline)) {
        constexpr int S6 = decltype(S_)::value;
        constexpr int S = S6 % 3;
        constexpr int D = (S + 2) % 3;          // the accumulator slot that completes
        constexpr int YW = (S6 + 1) & 1;        // ring slot written: intermediate row j - 3
        const int RS = (6 % PD == 0) ? S6 % PD : j % PD;
        if constexpr ((DBG & 32) != 0) {  // probe: two-row DMAs every other step, waited whole
            if constexpr (S6 % 2 == 0) rows_wait<0>();
        } else {
            rows_wait<VMW_B>();  // this wave's part of x row j has landed
        }
        if constexpr ((DBG & 16) == 0) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // + everyone's reads of the slots refilled
        if constexpr ((DBG & 32) != 0) {
            // probe (timing only): rows j + 2, j + 3 of every channel as ONE run of 2 x W floats per channel
            // (896 bytes at W = 112) instead of two 448-byte runs a step apart
            if constexpr (S6 % 2 == 0) {
                const int h = p0 + j;
                const bool hok = h + 1 < a.H;
                const uint32_t roff = (uint32_t)(hok ? h : 0) * (uint32_t)a.W * 4u;
                const uint32_t base = raw_lds + (uint32_t)((S6 / 2 % 2) * kPWRaw) + (uint32_t)(4 * sw) * 1024u;
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const int e = 64 * (8 * sw + i) + lane;  // float4 e of the [32][2 W / 4] pair
                    const int c = e / 56, q = 4 * (e - c * 56);
                    const uint32_t vo = (hok && c < CC) ? ((uint32_t)c * (uint32_t)HW + (uint32_t)q) * 4u + roff : 0x7fffffffu;
                    rows_dma16<(NTS & 2) != 0>(rs, vo, 0u, base + (uint32_t)(i & 3) * 1024u);
                }
            }
        } else if constexpr ((DBG & 2) == 0) {
            load_x((6 % PD == 0) ? (S6 + PD - 1) % PD : (j - 1 + PD) % PD, j - 1 + PD);
        }
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
        if constexpr ((DBG & 8) == 0) {  // epilogue 1: affine / activation, zeros outside the image (conv 2's padding), exact split
            const int i1 = j - 3;
            const int r1 = p0 - 1 + i1;
            const bool irow = i1 >= 0 && i1 < n1 && r1 >= 0 && r1 < a.H;
            const int p = lane & 15, g = lane >> 4;
            unsigned char* yw = yr + YW * yslot;
#pragma unroll
            for (int grp = 0; grp < NG; ++grp) {
                const int q = q0 + 16 * grp + p;  // lane: pixel q, channels 16 nt + 4 g .. + 3
                const bool okq = irow && q < a.W;
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) {
                    uint32_t b4[4];
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        float t;
                        if constexpr (E == 0) {
                            t = pend[grp][nt][e] * scale + 0.0f;
                        } else if constexpr (E == 2) {
                            const int c = nt * 4 + e;
                            t = pend[grp][nt][e] * es[c] + eb[c];  // folded affine, then ReLU
                            t = t < 0.0f ? 0.0f : t;
                        } else {
                            const int c = nt * 4 + e;
                            t = epi_act((pend[grp][nt][e] * scale + bk[c]) * es[c] + eb[c], a.act1);
                        }
                        b4[e] = okq ? __float_as_uint(t) : 0u;
                    }
                    uint2 h2, m2, l2;
                    split4p<false>(b4, h2, m2, l2);
                    const int wo = pw_oct(q + 1, (4 * nt + g) >> 1) + 8 * (g & 1);
                    *reinterpret_cast<uint2*>(yw + wo) = h2;
                    *reinterpret_cast<uint2*>(yw + YPL + wo) = m2;
                    *reinterpret_cast<uint2*>(yw + 2 * YPL + wo) = l2;
                }
            }
        }
        if constexpr ((DBG & 8) == 0) {  // the exact split of x row j into the strip's planes
            uint4 hi, mid, lo;
            split3<false>(bx[0], hi, mid, lo);
            *reinterpret_cast<uint4*>(slab + wa0) = hi;
            *reinterpret_cast<uint4*>(slab + PL + wa0) = mid;
            *reinterpret_cast<uint4*>(slab + 2 * PL + wa0) = lo;
            split3<false>(bx[1], hi, mid, lo);
            *reinterpret_cast<uint4*>(slab + wa1) = hi;
            *reinterpret_cast<uint4*>(slab + PL + wa1) = mid;
            *reinterpret_cast<uint4*>(slab + 2 * PL + wa1) = lo;
            uint16_t h16, m16, l16;
            split1(h_ok ? hx : 0u, h16, m16, l16);
            *reinterpret_cast<uint16_t*>(slab + wa_h) = h16;
            *reinterpret_cast<uint16_t*>(slab + PL + wa_h) = m16;
            *reinterpret_cast<uint16_t*>(slab + 2 * PL + wa_h) = l16;
        }
        if constexpr ((DBG & 1) == 0) {
            // x rows outside the image (the fill steps' padding rows, past the segment) are zeros: their
            // MFMAs would add exact zeros, so the wave skips them (wave-uniform) and only starts slot SL[0]
            const int h = p0 - 2 + j;
            if (j < nx && h >= 0 && h < a.H)
                mfmas(std::integral_constant<int, S>{}, std::true_type{}, slab);
            else
                zero_slot(std::integral_constant<int, S>{});
        }
#pragma unroll
        for (int grp = 0; grp < NG; ++grp)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) pend[grp][nt] = acc[D][grp][nt];
    };

    // ---- A, step j: conv 2 on intermediate row j - 4 (ring slot YR; unconditional: in the first steps it
    // reads the zeroed slots and its outputs are dropped), then epilogue 2 of output row j - 6: lane L holds
    // pixels 4g .. 4g + 3 of each group for channel 16 nt + (L & 15); one row_ror:8 DPP move per value
    // gives store A channels 0-7 and store B channels 8-15 of the tile as whole 128-byte runs
    auto stepA = [&](auto S_, int j) __attribute__((always_inline)) {
        constexpr int S6 = decltype(S_)::value;
        constexpr int S = S6 % 3;
        constexpr int D = (S + 2) % 3;
        constexpr int YR = S6 & 1;              // ring slot read: intermediate row j - 4
        const int RS = (6 % PD == 0) ? S6 % PD : j % PD;
        if constexpr (RES) rows_wait<VMW_A>();  // the residual of output row j - 6 has landed
        if constexpr ((DBG & 16) == 0) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // + B's epilogue-1 writes
        if constexpr (RES) load_res((6 % PD == 0) ? (S6 + PD - 1) % PD : (j - 1 + PD) % PD, j - 1 + PD);
        if constexpr ((DBG & 1) == 0) {
            // intermediate rows outside the image / segment were written as zeros by epilogue 1: skipped
            const int i2 = j - 4, r2 = p0 - 1 + i2;
            if (i2 >= 0 && i2 < n1 && r2 >= 0 && r2 < a.H)
                mfmas(std::integral_constant<int, S>{}, std::false_type{}, yr + YR * yslot);
            else
                zero_slot(std::integral_constant<int, S>{});
        }
        const int o = j - 6;
        const bool orow = o >= 0 && o < rbe;
        const unsigned char* rres_row = resr + RS * kPWRes;
        const int g = lane >> 4;
        const int qs = q0 + ((lane & 8) ? 16 : 0) + 4 * g;
        const uint32_t rowoff = (uint32_t)(orow ? p0 + o : 0) * a.W + (uint32_t)qs;
        const bool ok = orow && qs < a.W;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
            const int ch = 16 * nt + (lane & 15);
            floatx4 vv[NG];
#pragma unroll
            for (int grp = 0; grp < NG; ++grp) {
                floatx4 v;
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    v[e] = E == 0 ? acc[D][grp][nt][e] * scale + 0.0f
                           : E == 2 ? acc[D][grp][nt][e] * es[nt] + eb[nt]  // folded: scale2 * ps2, b2 * ps2 + pb2
                                    : (acc[D][grp][nt][e] * scale + bk[nt]) * es[nt] + eb[nt];
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
            if constexpr ((DBG & 32) != 0) {  // probe: both rows of a pair stored back to back, every other step
                if constexpr (S6 % 2 == 1) {
                    const uint32_t ro2 = rowoff >= (uint32_t)a.W ? rowoff - (uint32_t)a.W : rowoff;
                    rows_store<(NTS & 1) != 0>(ry, ok ? (ca * (uint32_t)HW + ro2) * 4u : 0x7fffffffu, sa);
                    rows_store<(NTS & 1) != 0>(ry, ok ? (ca * (uint32_t)HW + rowoff) * 4u : 0x7fffffffu, sa);
                    rows_store<(NTS & 1) != 0>(ry, ok ? (cb * (uint32_t)HW + ro2) * 4u : 0x7fffffffu, sb);
                    rows_store<(NTS & 1) != 0>(ry, ok ? (cb * (uint32_t)HW + rowoff) * 4u : 0x7fffffffu, sb);
                }
            } else if constexpr ((DBG & 4) == 0) {
                rows_store<(NTS & 1) != 0>(ry, ok ? (ca * (uint32_t)HW + rowoff) * 4u : 0x7fffffffu, sa);
                rows_store<(NTS & 1) != 0>(ry, ok ? (cb * (uint32_t)HW + rowoff) * 4u : 0x7fffffffu, sb);
            }
        }
    };

    // prologue DMAs: B x rows 0 .. PD-2; A (RES) the residual slots of steps 0 .. PD-2, each followed by
    // ST dropped stores (A's steady-state count)
    if (!roleA) {
#pragma unroll
        for (int r = 0; r < PD - 1; ++r) load_x(r, r);
    } else if constexpr (RES) {
        const floatx4 z = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int r = 0; r < PD - 1; ++r) {
            load_res(r, r);
#pragma unroll
            for (int i = 0; i < ST; ++i) rows_store<(NTS & 1) != 0>(ry, 0x7fffffffu, z);
        }
    }
    // ---- each wave quantizes + packs its conv's weights into VGPRs while those DMAs fly (the scale
    // reductions are block-wide; scratch: the intermediate planes, zeroed right after)
    {
        unsigned* red = reinterpret_cast<unsigned*>(yr);
        unsigned* thr = red + 16;
        uint4* fr = reinterpret_cast<uint4*>(yr + 4096);  // 2 x NF fragments (36 KB of the 50 KB planes)
        static_assert(4096 + 2 * NF * 64 * 16 <= 2 * yslot, "fragment scratch");
        bool fin1, fin2;
        const float scale1 = wq_prologue(a.q1, thr, red, 2 * kPWWaves, fin1);
        if constexpr ((DBG & 128) == 0) wq_pack_rows_lds<CC>(a.q1, CC, CC, NT, KS, scale1, fin1, thr, fr, NF);
        const float scale2 = wq_prologue(a.q2, thr, red, 2 * kPWWaves, fin2);
        if constexpr ((DBG & 128) == 0) {
            wq_pack_rows_lds<CC>(a.q2, CC, CC, NT, KS, scale2, fin2, thr, fr + NF * 64, NF);
            const uint4* frw = fr + (roleA ? NF * 64 : 0);
#pragma unroll
            for (int f = 0; f < NF; ++f) bw[f] = __builtin_bit_cast(bf16x8, frw[f * 64 + lane]);
        }
        scale = roleA ? scale2 : scale1;
        fin = roleA ? fin2 : fin1;
        if constexpr (E != 0) {
            const float *b = roleA ? a.b2 : a.b1, *ps = roleA ? a.ps2 : a.ps1, *pb = roleA ? a.pb2 : a.pb1;
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int k = roleA ? 16 * nt + (lane & 15) : 16 * nt + 4 * (lane >> 4) + e;
                    bk[nt * 4 + e] = b ? b[k] : 0.0f;
                    es[nt * 4 + e] = ps ? ps[k] : 1.0f;
                    eb[nt * 4 + e] = pb ? pb[k] : 0.0f;
                }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every staged value lands here
        if constexpr (E != 0) {
#pragma unroll
            for (int c = 0; c < NT * 4; ++c) asm volatile("" : "+v"(bk[c]), "+v"(es[c]), "+v"(eb[c]));
        }
#pragma unroll
        for (int f = 0; f < NF; ++f) asm volatile("" : "+v"(bw[f]));
        if constexpr (E == 2) {  // BasicBlock form: the conv scale and bias folded into the affine
#pragma unroll
            for (int c = 0; c < NT * 4; ++c) {
                eb[c] = bk[c] * es[c] + eb[c];
                es[c] = scale * es[c];
            }
        }
        // A's per-tile parameters sit at index nt * 4 (e = 0): move them to index nt
        if constexpr (E != 0) {
            if (roleA) {
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) {
                    bk[nt] = bk[nt * 4];
                    es[nt] = es[nt * 4];
                    eb[nt] = eb[nt * 4];
                }
            }
        }
        __syncthreads();  // scratch reads done: zero the intermediate planes (padding columns)
        for (int e = tid; e < (2 * yslot) / 16; e += blockDim.x)
            reinterpret_cast<uint4*>(yr)[e] = make_uint4(0u, 0u, 0u, 0u);
        // step 0's barrier publishes the zeros
    }
    (void)fin;
    if constexpr ((DBG & 64) != 0) return;  // probe: launch + weight staging only
    if (roleA) {
        for (int j = 0; j < nsteps; j += 6) {
            stepA(std::integral_constant<int, 0>{}, j);
            stepA(std::integral_constant<int, 1>{}, j + 1);
            stepA(std::integral_constant<int, 2>{}, j + 2);
            if (j + 3 >= nsteps) break;
            stepA(std::integral_constant<int, 3>{}, j + 3);
            stepA(std::integral_constant<int, 4>{}, j + 4);
            stepA(std::integral_constant<int, 5>{}, j + 5);
        }
    } else {
        for (int j = 0; j < nsteps; j += 6) {
            stepB(std::integral_constant<int, 0>{}, j);
            stepB(std::integral_constant<int, 1>{}, j + 1);
            stepB(std::integral_constant<int, 2>{}, j + 2);
            if (j + 3 >= nsteps) break;
            stepB(std::integral_constant<int, 3>{}, j + 3);
            stepB(std::integral_constant<int, 4>{}, j + 4);
            stepB(std::integral_constant<int, 5>{}, j + 5);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // trailing DMAs / stores land before the wave ends
}

namespace {

size_t pairw_lds(int pd, bool res) {
    return (size_t)pd * kPWRaw + 2 * 3 * (size_t)kPWYPL + (size_t)kPWWaves * 3 * kPWPL +
           (res ? (size_t)kPWWaves * pd * kPWRes : 0);
}

template <int PD, int NTS>
hipError_t launch_pairw_t(int blocks, size_t lds, const PairWArgs& a, const float* x, float* y, bool res, hipStream_t s) {
    const bool plain = !res && !a.b1 && !a.b2 && !a.ps1 && !a.pb1 && !a.ps2 && !a.pb2 && a.act1 == 0 && a.act2 == 0;
    const dim3 grid((unsigned)blocks), block(64 * 2 * kPWWaves);
#ifdef PO2Q_PAIRW_DIAG
    if (const char* dv = getenv("PO2Q_PAIR_W32_DBG")) {
        const int dbg = atoi(dv);
#define PO2Q_PWD(v) \
        if (dbg == v && plain && NTS == 3) { \
            hipLaunchKernelGGL((conv_pairw<PD, NTS, false, 0, v>), grid, block, lds, s, x, y, a); \
            return hipGetLastError(); \
        }
        PO2Q_PWD(9) PO2Q_PWD(11) PO2Q_PWD(13) PO2Q_PWD(15) PO2Q_PWD(25) PO2Q_PWD(29) PO2Q_PWD(27)
        PO2Q_PWD(31) PO2Q_PWD(64) PO2Q_PWD(192) PO2Q_PWD(128)
#undef PO2Q_PWD
    }
#endif
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

// PO2Q_PAIR_W32=0 turns the role-split kernel off (A/B and test knob: conv_pair<32> takes the shape);
// on by default: 0.305 vs 0.319 ms plain, 0.328 vs 0.351 block, bench 25.2k vs 24.8k img/s
// (profiles/r06_wpack_ab.jsonl).  PO2Q_PAIR_W32_NTS the store / load policy (default 3: non-temporal x
// loads and y stores)
int pairw_knob() {
    const char* e = getenv("PO2Q_PAIR_W32");
    return (e && e[0] == '0') ? 0 : 1;
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
    // x ring depth 2: depths 3 - 5 (plain form) measured the same (profiles/r06_pairw_ablation.jsonl, pd2-5)
    const int pd = 2;
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
    PO2Q_PW(2, 1)
#endif
#undef PO2Q_PW
    return hipErrorInvalidValue;
}

}  // namespace po2q
