// Two chained quantized 3x3 / stride-1 / pad-1 convs, C = 16 -> 16 -> 16, in ONE kernel:
//   y = act2(Q(w2) * act1(Q(w1) * x  [* ps1 + pb1]) [* ps2 + pb2] (+ res))
// -- the two QuantizedConv2d of a ResNet56 stage-1 BasicBlock (reference models/resnet.py:
// 55-71; each conv is QuantizedConv2d.forward, models/quantized_conv.py:32-38) with the
// block's eval BatchNorm / ReLU between and after them.  The intermediate activation never
// goes to HBM: a block keeps it as a 2-row fp32 ring in LDS, so a pair moves x in + y out
// (1.64 GB at bs = 256 @224) instead of twice that.
//
// Structure: the full-row-block kernel of po2q_conv_rowsf.hip (block = image x segment of
// RB output rows x the whole width, 7 waves of 32 columns, one s_barrier per step, whole-row
// LDS-DMA of x into a PD-slot raw ring, exact bf16x3 split into wave-private planes, row
// reuse over the 3 tap rows, hand-counted vmcnt), run twice per step:
//   step j:  wait for x row j (own DMAs), s_waitcnt lgkmcnt(0) + s_barrier, refill the slot
//            of x row j-1 (+ the residual row of the output stored PD-1 steps later);
//            conv 2 (j >= 3): split intermediate row j-3 from the shared ring (its halo
//            columns are the neighbours' part), MFMAs with w2, output row j-5 -> epilogue
//            2 -> transposed 128-byte-run stores;
//            conv 1: split x row j, MFMAs with w1, intermediate row j-2 -> epilogue 1 ->
//            the shared ring slot (j-2) & 1 (zeros outside the image: conv 2's padding).
// A segment recomputes two intermediate rows of its neighbours (RB + 2 conv-1 rows).
// Both weights are quantized + packed by the block itself (wq_* of po2q_quant_dev.h) into
// VGPRs: one launch per pair, no pack kernels.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdint>
#include <string>
#include <type_traits>
#ifdef PO2Q_PAIR_STAMPS
#include <cstdio>
#include <cstdlib>
#include <vector>
#endif

#include "../../include/po2q.h"
#include "po2q_epi.h"
#include "po2q_internal.h"
#include "po2q_quant_dev.h"
#include "po2q_rows_dev.h"
#include "po2q_x3_dev.h"

namespace po2q {

namespace {
template <int CC> constexpr int kQSW = 512 / CC;                              // output columns per wave
template <int CC> constexpr int kQPlane = (kQSW<CC> + 2) * 2 * CC + 32;      // x planes: [SW+2 px][CC] bf16 + zero slot
constexpr int kQResSlot = 2048;                                               // residual of a wave's strip and row
template <int CC> constexpr int kQKS = CC == 16 ? 2 : 3;                     // k-steps per tap row
}  // namespace

struct PairArgs {
    int N, H, W;      // P = H, Q = W
    int Wp;           // SW x waves
    int YPL;          // bytes of one shared intermediate plane: (Wp + 3) pixels x 2C bytes
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
    int prio;          // 1: the second wave of each SIMD (waves 4..) issues at priority 1
    unsigned* stamps;  // PO2Q_PAIR_STAMPS diagnostic builds only: per-wave phase cycle sums
    int mw;            // 1: the memory-wave kernel (MW) where it applies
};

// Diagnostic build (-DPO2Q_PAIR_STAMPS, `make pairstamps`): s_memtime phase stamps (guide "In-kernel
// stamps"; the sched_barriers serialize each phase, so read the shares, not the total); never in
// the product build.
#ifdef PO2Q_PAIR_STAMPS
#define PO2Q_PSTAMP(i)                                                                   \
    do {                                                                                 \
        __builtin_amdgcn_sched_barrier(0);                                               \
        unsigned long long t_;                                                           \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");        \
        __builtin_amdgcn_sched_barrier(0);                                               \
        ph_[i] += (unsigned)(t_ - tprev_);                                               \
        tprev_ = t_;                                                                     \
    } while (0)
#else
#define PO2Q_PSTAMP(i) \
    do {               \
    } while (0)
#endif

// Byte offset of the 16-byte channel octet `oc` (channels 8 oc .. 8 oc + 7) of pixel P in a
// shared intermediate plane ([pixel][C] bf16, 2C bytes per pixel), XOR-swizzled at octet
// granularity: conv 2's A-fragment reads are then ONE conflict-free ds_read_b128 per lane (the
// four 16-lane groups of that instruction hit 64 distinct banks), and conv 1's epilogue writes
// (ds_write_b64 of 4 channels, 16 contiguous lanes per group) are 2-way -- against two 2-way
// ds_read_b64 per fragment with the 8-byte-chunk swizzle this replaces (bank model of
// MI355X_MICROARCH.md "LDS"; PMC SQ_LDS_BANK_CONFLICT was 35 % of the pair's LDS cycles).
template <int CC>
__device__ __forceinline__ int yoct(int P, int oc) {
    return P * (2 * CC) + 16 * (oc ^ (CC == 16 ? ((P >> 2) & 1) : ((P >> 1) & 3)));
}

// Byte offset of channel octet `oc` of pixel hp in a wave's x planes.  C = 16: [pixel][16 ch]
// with the octet XOR-swizzled by (hp >> 2) & 1, so the split's ds_write_b128 (8 contiguous
// lanes = 8 consecutive pixels) covers all 32 banks and conv 1's fragment reads stay
// conflict-free (the unswizzled layout made every split write 2-way); C = 32: x_addr.
template <int CC>
__device__ __forceinline__ int xa(int hp, int oc) {
    if constexpr (CC == 16)
        return hp * 32 + 16 * (oc ^ ((hp >> 2) & 1));
    else
        return x_addr<CC>(hp, oc);
}

// The intermediate h lives in LDS already split: 2 ring slots x 3 planes (hi / mid / lo)
// x [Wp + 3 pixels][C ch] bf16, pixel index = column + 1 (pixel 0 and Wp + 1 are conv 2's
// zero padding columns, pixel Wp + 2 the zero slot of C = 16's k-step padding), shared by
// the block: conv 2 reads its A fragments -- halo columns included -- straight from it.
// Conv 1 runs in the transposed MFMA form (A = weights, B = x) so each lane holds 4
// consecutive channels of one pixel: its epilogue splits them and writes 8 bytes per plane.
// CC: 16 (7 waves of 32 columns at W = 224, weights in VGPRs) or 32 (7 waves of 16 columns
// at W = 112; conv 2's B fragments in LDS).  PD: x ring slots.  NTS bit 0: non-temporal
// stores, bit 1: non-temporal x loads.
// E: 0 = plain chain (no bias / affine / activation / residual: y = scale * acc), 1 = the
// general epilogues, 2 = the BasicBlock form (ReLU after both BNs: the conv scale and bias folded
// into the BN affine at staging, a compile-time ReLU; the kernel is bound by vector-instruction
// issue, so the common forms skip that work).
// (Measured off and removed in round 6, numbers in DESIGN.md: the stagger kernel -- waves 4.. one
// epilogue late --, packed-fp32 splits, conv 2's tap-row-0 weights in VGPRs at C = 32, a one-k-step
// fragment prefetch, temporal C = 32 stores, and the role-split kernel conv_pair_ab.)
// DBG (diagnostic builds only, -DPO2Q_PAIR_DIAG, PO2Q_PAIR_DEBUG; timing only, outputs are
// wrong): bit 1 no conv-2 MFMAs, 2 no conv-1 MFMAs, 4 no x DMAs, 8 no output stores, 16 no
// split / epilogue-1 plane writes.
// MW 1 (memory wave): an eighth wave issues every x DMA of the block, PD - 1 rows ahead, and joins
// the per-step barrier; the seven compute waves issue no loads, so they never wait on a vmcnt (their
// stores are never waited for until the end).  Without it each compute wave waits, every step, for
// its own x DMA of the previous step AND every store issued before it.  Plain / general forms
// without a residual, seven compute waves (C = 16: 192 < W <= 224, C = 32: 96 < W <= 112); a row is
// 14 DMA instructions either way (C x 7 * 512 / C / 4 float4).
template <int CC, int PD, int NTS, bool RES, int E = 1, int DBG = 0, int MW = 0>
__global__ __launch_bounds__(512, 1) void conv_pair(const float* __restrict__ x, float* __restrict__ y,
                                                    PairArgs a) {
    // MW with RES: the residual IS x (the BasicBlock's identity shortcut, checked on the host) and is
    // read from the x ring itself: raw row r is split at step r and re-read as output row r - 2's
    // residual at step r + 3, so the ring keeps 4 rows behind the current one (MWL = 4) -- no
    // residual DMAs at all.  Without RES the slot of row j - 1 is refilled at step j (MWL = 1).
    constexpr int MWL = RES ? 4 : 1;
    static_assert(!MW || PD - MWL - 1 >= 1, "memory wave: at least one row in flight");
    static_assert(CC == 16 || CC == 32, "C = 16 or 32");
    static_assert(PD >= 2 && PD <= 6, "raw ring slots");
    constexpr int SW = kQSW<CC>, WC = SW + 2, PL = kQPlane<CC>, KS = kQKS<CC>;
    constexpr int NG = SW / 16;   // 16-pixel groups per wave
    constexpr int NT = CC / 16;   // 16-channel output tiles (K = C)
    constexpr int NF = 3 * KS * NT;                 // B fragments per conv
    constexpr bool WL2 = CC == 32;                  // conv 2's B fragments in LDS (VGPR budget)
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nw = (int)(blockDim.x >> 6) - MW;  // compute waves (MW: wave nw is the memory wave)
    // bytes per channel row of the raw x ring.  MW at C = 16 pads each row by one float4: the row pitch is then
    // 4 dwords off a multiple of 32 banks, so the halo reads (one column, 8 / 16 channels per 32-lane
    // group) hit distinct banks instead of one (16-way at C = 16: SQ_LDS_BANK_CONFLICT)
    // (C = 16 only: at C = 32 the padded ring would not leave 5 slots in the LDS)
    constexpr bool RPAD = MW && CC == 16;
    const int RPB = a.Wp * 4 + (RPAD ? 16 : 0);
    // padded: a slot is whole 1 KiB DMA instructions (the last one's tail lanes load zeros past the
    // padded rows; they must land inside the slot)
    const int rawslot = RPAD ? (CC * RPB + 1023) / 1024 * 1024 : CC * RPB;
    // the intermediate planes are sized for the widest image (7 waves): a compile-time pitch turns
    // every slot / plane offset of the fragment reads and epilogue writes into an immediate
    constexpr int YPL = (7 * SW + 3) * 2 * CC;
    constexpr int yslot = 3 * YPL;
    unsigned char* raw = lds;                                   // PD x [C][Wp] fp32 (x rows)
    unsigned char* yr = raw + PD * rawslot;                     // 2 x 3 planes (intermediate, split)
    unsigned char* slab = yr + 2 * yslot + wave * (3 * PL);     // this wave's x planes
    unsigned char* resr = yr + 2 * yslot + nw * (3 * PL) + wave * (PD * kQResSlot);
    uint4* wl2 = reinterpret_cast<uint4*>(yr + 2 * yslot + nw * (3 * PL) + (RES ? nw * PD * kQResSlot : 0));
    const int zero_off = WC * CC * 2;
    constexpr int yzero = (7 * SW + 2) * (2 * CC);              // zero slot of a shared plane

    int blk = blockIdx.x;
    if (a.remap) blk = (blk & 7) * (int)(gridDim.x >> 3) + (blk >> 3);
    if (blk >= a.items) return;  // block-uniform
    const int seg = blk % a.nseg;
    const int n = blk / a.nseg;
    const int p0 = seg * a.RB;
    const int rbe = min(a.RB, a.H - p0);
    const int nx = rbe + 4;      // x rows p0-2 .. p0+rbe+1
    const int n1 = rbe + 2;      // intermediate rows p0-1 .. p0+rbe
    const int nsteps = nx + 1;   // output row p0 + o completes at step o + 5
    const int q0 = wave * SW;

    // ---- x DMA: lane l of this wave's instruction i -> float4 e = 64(2w + i) + l of the
    // row's C x Wp/4 float4 (whole-row runs; columns >= W read out of range: zeros)
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
    const __amdgpu_buffer_rsrc_t rres = rows_rsrc(RES ? a.res + (int64_t)n * CC * HW : x, RES ? CC * HW * 4 : 4);
    uint32_t vr[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int e = 64 * i + lane;
        const int c = e / (SW / 4), q = q0 + 4 * (e % (SW / 4));
        vr[i] = q < a.W ? ((uint32_t)c * (uint32_t)HW + (uint32_t)q) * 4u : 0x7fffffffu;
    }
    const uint32_t res_lds = (uint32_t)(uintptr_t)resr;
    // x row jn into raw slot sl; with RES the residual of the output row stored at step jn
    auto load_row = [&](int sl, int jn) __attribute__((always_inline)) {
        if constexpr ((DBG & 4) != 0) return;
        const int h = p0 - 2 + jn;
        const bool hok = jn < nx && h >= 0 && h < a.H;
        const uint32_t roff = (uint32_t)(hok ? h : 0) * (uint32_t)a.W * 4u;
        const uint32_t base = raw_lds + (uint32_t)(sl * rawslot) + (uint32_t)(2 * wave) * 1024u;
#pragma unroll
        for (int i = 0; i < 2; ++i)
            rows_dma16<(NTS & 2) != 0>(rs, (hok && vi[i] != 0x7fffffffu) ? vi[i] + roff : 0x7fffffffu, 0u, base + i * 1024u);
        if constexpr (RES) {
            const int o = jn - 5;
            const bool ook = jn >= 5 && o < rbe;
            const uint32_t ooff = (uint32_t)(ook ? p0 + o : 0) * (uint32_t)a.W * 4u;
#pragma unroll
            for (int i = 0; i < 2; ++i)
                rows_dma16<false>(rres, (ook && vr[i] != 0x7fffffffu) ? vr[i] + ooff : 0x7fffffffu, 0u,
                                  res_lds + (uint32_t)(sl * kQResSlot) + i * 1024u);
        }
    };

    // ---- x split: lane -> (column sc of the strip, channel octet so); halo lanes < 2C ->
    // (side, channel) from the neighbours' columns of the shared raw row (zero outside)
    const int sc = lane % SW, so = lane / SW;
    const int wa_i = xa<CC>(sc + 1, so);
    // Each 32-lane group (one LDS cycle of ds_read_b32) reads C / 2 channels of both halo columns:
    // group g takes channels (C / 2) g .. + C / 2 - 1, its lane l -> side (l % C) / (C / 2); at C = 16
    // lanes 16-31 of a group repeat lanes 0-15 (same values to the same addresses: no divergent branch)
    const int hl = lane % CC;
    const int hside = hl / (CC / 2), hch = (CC / 2) * (lane >> 5) + hl % (CC / 2);
    const int hq = hside ? q0 + SW : q0 - 1;
    const bool h_ok = hq >= 0 && hq < a.W;
    const int wa_h = xa<CC>(hside ? WC - 1 : 0, hch >> 3) + (hch & 7) * 2;
    const int rdx0 = (so * 8) * RPB + (q0 + sc) * 4;
    const int rdx_h = hch * RPB + (h_ok ? hq : 0) * 4;
    // A fragment addresses: x planes (wave-private, pixel = strip column + 1) and shared
    // intermediate planes (pixel = column + 1, swizzled octet o): one b128 each
    // C = 16 pairs the s2 tap of two planes in one k-step: per halo row and group the k-steps are
    // (s0 | s1) of each plane, (s2 hi | s2 mid) and (s2 lo | zero) -- 5 MFMAs per tap row where
    // (s2 | zero) per plane took 6 (the 9 16-channel units of a row fill 4.5 k-steps).  Lanes of
    // k-half 1 (g >= 2) of the paired fragment read the mid plane, so its offset carries the plane:
    // aoff[grp][1] / yoff[grp][1] = (s2 hi | s2 mid), aoff2 / yoff2 = (s2 lo | zero slot).
    int aoff[NG][KS], yoff[NG][KS], aoff2[NG], yoff2[NG];
    {
        const int p = lane & 15, g = lane >> 4;
#pragma unroll
        for (int grp = 0; grp < NG; ++grp) {
            const int qc = q0 + 16 * grp + p;  // output column
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                if constexpr (CC == 16) {  // ks 0: taps (s0 | s1) x 16 ch; ks 1: the paired s2 fragments
                    const int xp = 16 * grp + p + (ks == 0 ? (g >> 1) : 2);
                    const int yp = qc + (ks == 0 ? (g >> 1) : 2);
                    const int o = g & 1;
                    if (ks == 0) {
                        aoff[grp][ks] = xa<CC>(xp, o);
                        yoff[grp][ks] = yoct<CC>(yp, o);
                    } else {
                        aoff[grp][ks] = xa<CC>(xp, o) + (g >= 2 ? PL : 0);
                        yoff[grp][ks] = yoct<CC>(yp, o) + (g >= 2 ? YPL : 0);
                        aoff2[grp] = g >= 2 ? zero_off : xa<CC>(xp, o) + 2 * PL;
                        yoff2[grp] = g >= 2 ? yzero : yoct<CC>(yp, o) + 2 * YPL;
                    }
                } else {  // ks = tap s, k = the 32 channels (octet g)
                    aoff[grp][ks] = xa<CC>(16 * grp + p + ks, g);
                    yoff[grp][ks] = yoct<CC>(qc + ks, g);
                    aoff2[grp] = yoff2[grp] = 0;
                }
            }
        }
    }

    const __amdgpu_buffer_rsrc_t ry = rows_rsrc(y + (int64_t)n * CC * HW, CC * HW * 4);
    constexpr int ST = NG * NT;               // stores per step (issued every step; dropped ones out of range)
    constexpr int LD = RES ? 4 : 2;           // DMAs per step
    constexpr int VMW = ST + (PD - 2) * (LD + ST);

    float scale1 = 1.0f, scale2 = 1.0f;
    bool fin1 = true, fin2 = true;
    bf16x8 bw1[NF], bw2[WL2 ? 1 : NF];
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
    // 3 tap rows x KS k-steps x 3 planes x NG groups x NT tiles of MFMAs on one split row
    // into accumulator slots SL.  TR (conv 1): transposed (A = weights), x planes, VGPR
    // weights; else (conv 2): shared planes (two b64 per fragment), weights per WL2
    auto mfmas = [&](auto S_, auto TR_, floatx4 (&acc)[3][NG][NT], const bf16x8 (&bw)[NF],
                     const bf16x8 (&bw2v)[WL2 ? 1 : NF], const unsigned char* pb) __attribute__((always_inline)) {
        constexpr int SR = decltype(S_)::value;
        constexpr bool TR = decltype(TR_)::value;
        constexpr int SL[3] = {(SR + 1) % 3, SR, (SR + 2) % 3};
        // fragments of k-step ks: the 3 planes, or for C = 16's k-step 1 the two paired ones; at
        // C = 32 (conv 2) also the 3 x NT B fragments of the k-step from LDS
        auto load_a = [&](int ks, bf16x8 (&af)[3][NG]) __attribute__((always_inline)) {
            const int np = (CC == 16 && ks == 1) ? 2 : 3;
#pragma unroll
            for (int pl = 0; pl < 3; ++pl)
#pragma unroll
                for (int grp = 0; grp < NG; ++grp) {
                    if (pl >= np) continue;
                    int off;
                    if (CC == 16 && ks == 1)
                        off = pl == 0 ? (TR ? aoff[grp][1] : yoff[grp][1]) : (TR ? aoff2[grp] : yoff2[grp]);
                    else
                        off = TR ? pl * PL + aoff[grp][ks] : pl * YPL + yoff[grp][ks];
                    af[pl][grp] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(pb + off));
                }
        };
        auto load_b = [&](int ks, bf16x8 (&bf)[3][NT]) __attribute__((always_inline)) {
#pragma unroll
            for (int r3 = 0; r3 < 3; ++r3)
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) {
                    const int rr = 2 - r3;
                    const int f = (rr * KS + ks) * NT + nt;
                    if constexpr (TR)
                        bf[r3][nt] = bw[f];
                    else if constexpr (WL2)
                        bf[r3][nt] = __builtin_bit_cast(bf16x8, wl2[f * 64 + lane]);
                    else
                        bf[r3][nt] = bw2v[WL2 ? 0 : f];
                }
        };
        auto mma = [&](int ks, const bf16x8 (&af)[3][NG], const bf16x8 (&bf)[3][NT]) __attribute__((always_inline)) {
            const int np = (CC == 16 && ks == 1) ? 2 : 3;
            // tap row 2 first: it feeds the slot that completes this step, so its epilogue can
            // start while the other tap rows' MFMAs of the last k-step still run
#pragma unroll
            for (int r3 = 0; r3 < 3; ++r3)
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) {
                    const int rr = 2 - r3;
                    const bf16x8 b = bf[r3][nt];
#pragma unroll
                    for (int pl = 0; pl < 3; ++pl)
#pragma unroll
                        for (int grp = 0; grp < NG; ++grp) {
                            if (pl >= np) continue;
                            // slot SL[0] (output row j + 1) starts at this step: its first MFMA takes a
                            // zero accumulator, so the epilogues need not clear the slot they retire
                            const floatx4 c = (rr == 0 && ks == 0 && pl == 0) ? floatx4{0.f, 0.f, 0.f, 0.f}
                                                                             : acc[SL[rr]][grp][nt];
                            acc[SL[rr]][grp][nt] = TR ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, af[pl][grp], c, 0, 0, 0)
                                                      : __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[pl][grp], b, c, 0, 0, 0);
                        }
                }
        };
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            bf16x8 af[3][NG], bf[3][NT];
            load_a(ks, af);
            load_b(ks, bf);
            mma(ks, af, bf);
        }
    };

    // conv-2 epilogue of the output row that completes at step j (accumulator slot D of S6)
    auto epi2 = [&](auto S_, int j) __attribute__((always_inline)) {
        constexpr int S6 = decltype(S_)::value;
        constexpr int D = (S6 % 3 + 2) % 3;
        const int RS = (6 % PD == 0) ? S6 % PD : j % PD;
        const int o = j - 5;
        const bool orow = o >= 0 && o < rbe;
        const unsigned char* rres_row = resr + RS * kQResSlot;  // loaded with x row j
        // MW: x row j - 3 (= image row p0 + o) still in the ring, [C][Wp] fp32
        const unsigned char* rres_ring = raw + ((j + PD - 3) % PD) * rawslot + q0 * 4;
        const int g = lane >> 4;
        floatx4 vv[NT][NG];
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
            const int ch = 16 * nt + (lane & 15);
            const uint32_t yrow = (uint32_t)ch * (uint32_t)HW + (uint32_t)(orow ? p0 + o : 0) * a.W;
#pragma unroll
            for (int grp = 0; grp < NG; ++grp) {
                const int ql = 16 * grp + 4 * g;  // strip column of the lane's 4 pixels
                floatx4 v;
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    v[e] = E == 0 ? acc2[D][grp][nt][e] * scale2 + 0.0f
                           : E == 2 ? acc2[D][grp][nt][e] * e2s[nt] + e2b[nt]  // folded: scale2 * ps2, b2 * ps2 + pb2
                                    : (acc2[D][grp][nt][e] * scale2 + bk2[nt]) * e2s[nt] + e2b[nt];
                if constexpr (RES) {
                    const floatx4 r = MW ? *reinterpret_cast<const floatx4*>(rres_ring + ch * RPB + ql * 4)
                                         : *reinterpret_cast<const floatx4*>(rres_row + ch * (SW * 4) + ql * 4);
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
                vv[nt][grp] = v;
                if constexpr (CC != 16) {
                    const int q = q0 + ql;
                    rows_store<(NTS & 1) != 0>(ry, (orow && q < a.W) ? (yrow + (uint32_t)q) * 4u : 0x7fffffffu, v);
                }
            }
        }
        if constexpr (CC == 16) {
            // Whole 128-byte lines per store: lane L holds pixels 4g .. 4g + 3 (vv[0][0]) and
            // 16 + 4g .. (vv[0][1]) of channel L & 15.  One row_ror:8 DPP exchange within each
            // 16-lane row gives store A channels 0-7 (lanes with bit 3 set take channel L & 7's
            // second half from lane L - 8) and store B channels 8-15 (lanes without it take
            // channel 8 + (L & 7)'s first half from lane L + 8): 8 lanes x 16 bytes = one full
            // line per channel, where two 64-byte halves from two stores cost partial-line
            // writes (PMC: 1.32x the output bytes with non-temporal stores).
            // One DPP move per value: the bank mask restricts the row_ror:8 write to the lanes that
            // take the other half (banks 2-3 = lanes 8-15 for store A, banks 0-1 for store B), the
            // others keep `old` -- no zero-initialised temporary and no select.
            const bool hi8 = (lane & 8) != 0;
            floatx4 sa, sb;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                sa[e] = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(vv[0][0][e]),
                                                                   __float_as_int(vv[0][NG - 1][e]), 0x128, 0xf, 0xc, false));
                sb[e] = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(vv[0][NG - 1][e]),
                                                                   __float_as_int(vv[0][0][e]), 0x128, 0xf, 0x3, false));
            }
            const int q = q0 + (hi8 ? 16 : 0) + 4 * g;
            const uint32_t rowoff = (uint32_t)(orow ? p0 + o : 0) * a.W + (uint32_t)q;
            const uint32_t ca = (uint32_t)(lane & 7), cb = 8u + (uint32_t)(lane & 7);
            const bool ok = orow && q < a.W;
            if constexpr ((DBG & 8) == 0) {
                rows_store<(NTS & 1) != 0>(ry, ok ? (ca * (uint32_t)HW + rowoff) * 4u : 0x7fffffffu, sa);
                rows_store<(NTS & 1) != 0>(ry, ok ? (cb * (uint32_t)HW + rowoff) * 4u : 0x7fffffffu, sb);
            }
        }
    };

    // exact split of x row j (8 channels of one strip column per lane + the halo lanes) into
    // this wave's planes
    auto split_x = [&](const uint32_t (&bx)[8], uint32_t hx) __attribute__((always_inline)) {
        if constexpr ((DBG & 16) != 0) return;
        uint4 hi, mid, lo;
        split3<false>(bx, hi, mid, lo);
        *reinterpret_cast<uint4*>(slab + wa_i) = hi;
        *reinterpret_cast<uint4*>(slab + PL + wa_i) = mid;
        *reinterpret_cast<uint4*>(slab + 2 * PL + wa_i) = lo;
        {
            uint16_t h16, m16, l16;
            split1(h_ok ? hx : 0u, h16, m16, l16);
            *reinterpret_cast<uint16_t*>(slab + wa_h) = h16;
            *reinterpret_cast<uint16_t*>(slab + PL + wa_h) = m16;
            *reinterpret_cast<uint16_t*>(slab + 2 * PL + wa_h) = l16;
        }
    };

    const bool strip_full = q0 + SW <= a.W;  // wave-uniform
#ifdef PO2Q_PAIR_STAMPS
    unsigned ph_[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long tprev_ = 0;
#endif

    auto step = [&](auto S_, int j) __attribute__((always_inline)) {
        constexpr int S6 = decltype(S_)::value;
        constexpr int S = S6 % 3;
        constexpr int D = (S + 2) % 3;          // the accumulator slot that completes
        constexpr int YW = S6 & 1;              // ring slot written: intermediate row j-2
        constexpr int YR = (S6 + 1) & 1;        // ring slot read: intermediate row j-3
        const int RS = (6 % PD == 0) ? S6 % PD : j % PD;
        PO2Q_PSTAMP(0);
        if constexpr (!MW) rows_wait<VMW>();  // this wave's part of x row j has landed
        PO2Q_PSTAMP(1);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // + everyone's plane writes
        PO2Q_PSTAMP(2);
        if constexpr (!MW) load_row((6 % PD == 0) ? (S6 + PD - 1) % PD : (j - 1 + PD) % PD, j - 1 + PD);
        // the x split's LDS reads next: their latency runs under conv 2's MFMAs
        uint32_t bx[8], hx;
        {
            const unsigned char* rw = raw + RS * rawslot;
#pragma unroll
            for (int e = 0; e < 8; ++e) bx[e] = *reinterpret_cast<const uint32_t*>(rw + rdx0 + e * RPB);
            hx = *reinterpret_cast<const uint32_t*>(rw + rdx_h);
        }

        // ---- conv 2 on intermediate row i = j - 3 (its halo index), straight from the shared planes
        // (unconditional: in steps 0-2 it reads the zeroed ring slots and its outputs are dropped --
        // no branch, so its MFMAs interleave with the epilogue-2 and x-split vector work below)
        if constexpr ((DBG & 1) == 0)
            mfmas(std::integral_constant<int, S>{}, std::false_type{}, acc2, bw1, bw2, yr + YR * yslot);
        PO2Q_PSTAMP(3);
        epi2(S_, j);
        PO2Q_PSTAMP(4);
        split_x(bx, hx);
        PO2Q_PSTAMP(5);

        // ---- conv 1 on x row j (transposed MFMAs); intermediate row i = j - 2 completes
        if constexpr ((DBG & 2) == 0) mfmas(std::integral_constant<int, S>{}, std::true_type{}, acc1, bw1, bw2, slab);
        PO2Q_PSTAMP(6);
        if constexpr ((DBG & 16) == 0) {
            const int i = j - 2;
            const int r1 = p0 - 1 + i;
            const bool irow = i >= 0 && i < n1 && r1 >= 0 && r1 < a.H;
            const int p = lane & 15, g = lane >> 4;
            unsigned char* yw = yr + YW * yslot;
            // wave-uniform: an image row whose every strip column is inside the image needs no
            // per-value select (the common case: W a multiple of the strip width)
            const bool allok = irow && strip_full;
#pragma unroll
            for (int grp = 0; grp < NG; ++grp) {
                const int q = q0 + 16 * grp + p;  // lane: pixel q, channels 16 nt + 4 g .. + 3
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) {
                    uint32_t b4[4];
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        float t;
                        if constexpr (E == 0) {
                            t = acc1[D][grp][nt][e] * scale1 + 0.0f;
                        } else if constexpr (E == 2) {
                            const int c = nt * 4 + e;
                            t = acc1[D][grp][nt][e] * e1s[c] + e1b[c];  // folded affine, then ReLU
                            t = t < 0.0f ? 0.0f : t;
                        } else {
                            const int c = nt * 4 + e;
                            t = epi_act((acc1[D][grp][nt][e] * scale1 + bk1[c]) * e1s[c] + e1b[c], a.act1);
                        }
                        b4[e] = __float_as_uint(t);
                    }
                    if (!allok) {  // wave-uniform: only rows / strips that leave the image pay the select
                        const bool ok = irow && q < a.W;
#pragma unroll
                        for (int e = 0; e < 4; ++e) b4[e] = ok ? b4[e] : 0u;
                    }
                    uint2 h2, m2, l2;
                    split4p<false>(b4, h2, m2, l2);
                    const int wo = yoct<CC>(q + 1, (4 * nt + g) >> 1) + 8 * (g & 1);
                    *reinterpret_cast<uint2*>(yw + wo) = h2;
                    *reinterpret_cast<uint2*>(yw + YPL + wo) = m2;
                    *reinterpret_cast<uint2*>(yw + 2 * YPL + wo) = l2;
                }
            }
        }
        PO2Q_PSTAMP(7);
#ifdef PO2Q_PAIR_STAMPS
        ph_[8] += 1;
#endif
    };

    // MW: the memory wave's DMA of x row jn into its raw ring slot: every float4 of the row's C x (Wp/4 + 1)
    // padded layout (instruction i, lane l -> float4 64 i + l; the pad float4 of each channel row and the
    // tail past C rows load out of range, i.e. zeros).  MWD instructions (15 where 14 covered the
    // unpadded row; MW runs 7 compute waves only: Wp = 7 x 512 / C)
    constexpr int MWW4 = 7 * SW / 4 + (RPAD ? 1 : 0);  // float4 per (padded) channel row
    constexpr int MWD = (CC * MWW4 + 63) / 64;
    auto mw_row = [&](int jn) __attribute__((always_inline)) {
        const int h = p0 - 2 + jn;
        const bool hok = jn < nx && h >= 0 && h < a.H;
        const uint32_t roff = (uint32_t)(hok ? h : 0) * (uint32_t)a.W * 4u;
        const uint32_t base = raw_lds + (uint32_t)((jn % PD) * rawslot);
#pragma unroll
        for (int i = 0; i < MWD; ++i) {
            const int e = 64 * i + lane;
            const int c = e / MWW4, q = 4 * (e - c * MWW4);
            const uint32_t vo = (hok && c < CC && q < a.W) ? ((uint32_t)c * (uint32_t)HW + (uint32_t)q) * 4u + roff
                                                            : 0x7fffffffu;
            rows_dma16<(NTS & 2) != 0>(rs, vo, 0u, base + (uint32_t)i * 1024u);
        }
    };
    if constexpr (MW) {
        if (wave == nw) {
#pragma unroll
            for (int r = 0; r < PD - MWL; ++r) mw_row(r);
        }
    } else {
        // x rows 0 .. PD-2, each followed by ST dropped stores (the steady-state count)
        const floatx4 z = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int r = 0; r < PD - 1; ++r) {
            load_row(r, r);
#pragma unroll
            for (int i = 0; i < ST; ++i) rows_store<(NTS & 1) != 0>(ry, 0x7fffffffu, z);
        }
    }
    // ---- both weights quantized + packed (VGPRs; conv 2's in LDS for C = 32) while those
    // DMAs fly (scratch: the intermediate planes, zeroed right after)
    {
        unsigned* red = reinterpret_cast<unsigned*>(yr);
        unsigned* thr = red + 16;
        uint4* fr = reinterpret_cast<uint4*>(yr + 4096);  // conv 1's fragments (and conv 2's for C = 16)
        static_assert(4096 + (WL2 ? 1 : 2) * NF * 64 * 16 <= 2 * yslot, "fragment scratch");
        scale1 = wq_prologue(a.q1, thr, red, nw + MW, fin1);
        wq_pack_rows_lds<CC>(a.q1, CC, CC, NT, KS, scale1, fin1, thr, fr, NF, CC == 16);
        scale2 = wq_prologue(a.q2, thr, red, nw + MW, fin2);
        if constexpr (WL2) {
            wq_pack_rows_lds<CC>(a.q2, CC, CC, NT, KS, scale2, fin2, thr, wl2, NF);
        } else {
            wq_pack_rows_lds<CC>(a.q2, CC, CC, NT, KS, scale2, fin2, thr, fr + NF * 64, NF, CC == 16);
#pragma unroll
            for (int f = 0; f < NF; ++f) bw2[WL2 ? 0 : f] = __builtin_bit_cast(bf16x8, fr[NF * 64 + f * 64 + lane]);
        }
#pragma unroll
        for (int f = 0; f < NF; ++f) bw1[f] = __builtin_bit_cast(bf16x8, fr[f * 64 + lane]);
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
        for (int f = 0; f < NF; ++f) asm volatile("" : "+v"(bw1[f]));
        if constexpr (!WL2) {
#pragma unroll
            for (int f = 0; f < NF; ++f) asm volatile("" : "+v"(bw2[WL2 ? 0 : f]));
        }
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
        __syncthreads();  // scratch reads done: zero the intermediate planes (padding columns, zero slots)
        for (int e = tid; e < (2 * yslot) / 16; e += blockDim.x)
            reinterpret_cast<uint4*>(yr)[e] = make_uint4(0u, 0u, 0u, 0u);
        if (lane < 3 && wave < nw)  // MW: the memory wave has no planes (wave nw's would be wl2 / beyond)
            *reinterpret_cast<uint4*>(slab + lane * PL + zero_off) = make_uint4(0u, 0u, 0u, 0u);
        // step 0's barrier publishes the zeros (and wl2)
    }
    // static priority for the younger wave of each SIMD (MI355X_MICROARCH two-waves item 4)
    if (a.prio && wave >= 4) __builtin_amdgcn_s_setprio(1);
#ifdef PO2Q_PAIR_STAMPS
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(tprev_)::"memory");
#endif
    if constexpr (MW) {
        if (wave == nw) {
            // the memory wave: before barrier j row j has landed (its DMA is the oldest of the PD - 1
            // rows in flight), after it the slot of row j - 1 (read by the splits of step j - 1, which
            // every wave finished before the barrier) takes row j + PD - 1.  Same barrier count as the
            // compute waves' loop.
            auto mstep = [&](int j) __attribute__((always_inline)) {
                rows_wait<MWD * (PD - MWL - 1)>();  // row j landed (rows j + 1 .. j + PD - MWL - 1 may fly)
                asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
                mw_row(j + PD - MWL);  // into the slot of row j - MWL, whose last reader was step j - 1
            };
            for (int j = 0; j < nsteps; j += 6) {
                mstep(j);
                mstep(j + 1);
                mstep(j + 2);
                if (j + 3 >= nsteps) break;
                mstep(j + 3);
                mstep(j + 4);
                mstep(j + 5);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            return;
        }
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
#ifdef PO2Q_PAIR_STAMPS
    if (lane == 0 && a.stamps)
        for (int i = 0; i < 9; ++i) a.stamps[((size_t)blockIdx.x * 8 + wave) * 9 + i] = ph_[i];
#endif
}


// ------------------------------------------------------------------ planning --
struct PairPlan {
    int C = 0, waves = 0, pd = 0, nts = 0, RB = 0, nseg = 0;
    int64_t blocks = 0;
    size_t lds = 0;
};

// RS (C = 16, seven 32-column strips, no residual): the stage-1 pair with its two convs given to
// different waves, as conv_pairw does at stage 2 -- waves 0-6 ("B") run conv 1 of strip w (their x DMAs,
// the exact split, conv 1's MFMAs, the conv-1 epilogue one step later into the shared intermediate
// ring), waves 7-13 ("A") run conv 2 of strip w - 7 on that ring and its epilogue with the stores.  A
// wave's chain per step is one conv instead of both, and 14 waves give each SIMD 3-4 of them to
// interleave.  Same fragments, same MFMA order per accumulator and the same epilogue expressions as
// conv_pair<16>: the same bits.
template <int PD, int NTS, int E>
__global__ __launch_bounds__(896, 1) void conv_pair_rs16(const float* __restrict__ x, float* __restrict__ y,
                                                         PairArgs a) {
    static_assert(PD >= 2 && PD <= 4, "raw ring slots");  // the product instantiates PD 3
    constexpr int CC = 16, SW = kQSW<16>, WC = SW + 2, PL = kQPlane<16>, KS = kQKS<16>;
    constexpr int NG = SW / 16, NT = 1, NF = 3 * KS * NT, NWR = 7;
    constexpr int YPL = (7 * SW + 3) * 2 * CC;
    constexpr int yslot = 3 * YPL;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool roleA = wave >= NWR;  // wave-uniform: conv 2 (A) or conv 1 (B)
    const int sw = roleA ? wave - NWR : wave;
    const int RPB = a.Wp * 4;
    const int rawslot = CC * RPB;
    unsigned char* raw = lds;                                // PD x [C][Wp] fp32
    unsigned char* yr = raw + PD * rawslot;                  // 2 x 3 planes (intermediate, split)
    unsigned char* slab = yr + 2 * yslot + sw * (3 * PL);    // B: its strip's x planes
    const int zero_off = WC * CC * 2;
    constexpr int yzero = (7 * SW + 2) * (2 * CC);

    int blk = blockIdx.x;
    if (a.remap) blk = (blk & 7) * (int)(gridDim.x >> 3) + (blk >> 3);
    if (blk >= a.items) return;  // block-uniform
    const int seg = blk % a.nseg;
    const int n = blk / a.nseg;
    const int p0 = seg * a.RB;
    const int rbe = min(a.RB, a.H - p0);
    const int nx = rbe + 4;   // x rows p0-2 .. p0+rbe+1
    const int n1 = rbe + 2;   // intermediate rows p0-1 .. p0+rbe
    const int nsteps = nx + 2;  // output row p0 + o completes at step o + 6
    const int q0 = sw * SW;
    const int HW = a.H * a.W;

    // ---- B: x DMA, conv_pair's mapping (lane l of instruction i -> float4 64(2 sw + i) + l of the row)
    const __amdgpu_buffer_rsrc_t rs = rows_rsrc(x + (int64_t)n * CC * HW, CC * HW * 4);
    const int W4 = a.Wp >> 2;
    uint32_t vi[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int e = 64 * (2 * sw + i) + lane;
        const int c = e / W4, q = 4 * (e - c * W4);
        vi[i] = q < a.W ? ((uint32_t)c * (uint32_t)HW + (uint32_t)q) * 4u : 0x7fffffffu;
    }
    const uint32_t raw_lds = (uint32_t)(uintptr_t)raw;
    auto load_x = [&](int sl, int jn) __attribute__((always_inline)) {
        const int h = p0 - 2 + jn;
        const bool hok = jn < nx && h >= 0 && h < a.H;
        const uint32_t roff = (uint32_t)(hok ? h : 0) * (uint32_t)a.W * 4u;
        const uint32_t base = raw_lds + (uint32_t)(sl * rawslot) + (uint32_t)(2 * sw) * 1024u;
#pragma unroll
        for (int i = 0; i < 2; ++i)
            rows_dma16<(NTS & 2) != 0>(rs, (hok && vi[i] != 0x7fffffffu) ? vi[i] + roff : 0x7fffffffu, 0u, base + i * 1024u);
    };
    // ---- B: the split (conv_pair's split_x lanes: column sc, octet so; halo lanes)
    const int sc = lane % SW, so = lane / SW;
    const int wa_i = xa<CC>(sc + 1, so);
    const int hl = lane % CC;
    const int hside = hl / (CC / 2), hch = (CC / 2) * (lane >> 5) + hl % (CC / 2);
    const int hq = hside ? q0 + SW : q0 - 1;
    const bool h_ok = hq >= 0 && hq < a.W;
    const int wa_h = xa<CC>(hside ? WC - 1 : 0, hch >> 3) + (hch & 7) * 2;
    const int rdx0 = (so * 8) * RPB + (q0 + sc) * 4;
    const int rdx_h = hch * RPB + (h_ok ? hq : 0) * 4;
    // fragment offsets: conv_pair's (B: x planes, A: the shared intermediate planes)
    int aoff[NG][KS], aoff2[NG];
    {
        const int p = lane & 15, g = lane >> 4;
#pragma unroll
        for (int grp = 0; grp < NG; ++grp) {
            const int qc = q0 + 16 * grp + p;
            const int o = g & 1;
            if (!roleA) {
                aoff[grp][0] = xa<CC>(16 * grp + p + (g >> 1), o);
                aoff[grp][1] = xa<CC>(16 * grp + p + 2, o) + (g >= 2 ? PL : 0);
                aoff2[grp] = g >= 2 ? zero_off : xa<CC>(16 * grp + p + 2, o) + 2 * PL;
            } else {
                aoff[grp][0] = yoct<CC>(qc + (g >> 1), o);
                aoff[grp][1] = yoct<CC>(qc + 2, o) + (g >= 2 ? YPL : 0);
                aoff2[grp] = g >= 2 ? yzero : yoct<CC>(qc + 2, o) + 2 * YPL;
            }
        }
    }
    const __amdgpu_buffer_rsrc_t ry = rows_rsrc(y + (int64_t)n * CC * HW, CC * HW * 4);
    constexpr int VMW_B = 2 * (PD - 2);  // B: its DMAs of the PD - 2 rows issued after row j's

    float scale = 1.0f;
    bool fin = true;
    bf16x8 bw[NF];
    float bk[E ? NT * 4 : 1], es[E ? NT * 4 : 1], eb[E ? NT * 4 : 1];  // B: ch 4 (lane >> 4) + e; A: index 0
    floatx4 acc[3][NG][NT];
#pragma unroll
    for (int sl = 0; sl < 3; ++sl)
#pragma unroll
        for (int grp = 0; grp < NG; ++grp) acc[sl][grp][0] = floatx4{0.f, 0.f, 0.f, 0.f};

    // conv_pair's mfmas for one conv: per k-step the planes' fragments (k-step 1: the paired s2 ones),
    // tap row 2 first, per accumulator k-step major, plane minor
    auto mfmas = [&](auto S_, auto TR_, const unsigned char* pb) __attribute__((always_inline)) {
        constexpr int SR = decltype(S_)::value;
        constexpr bool TR = decltype(TR_)::value;
        constexpr int SL[3] = {(SR + 1) % 3, SR, (SR + 2) % 3};
        constexpr int PLS = TR ? PL : YPL;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const int np = ks == 1 ? 2 : 3;
            bf16x8 af[3][NG];
#pragma unroll
            for (int pl = 0; pl < 3; ++pl)
#pragma unroll
                for (int grp = 0; grp < NG; ++grp) {
                    if (pl >= np) continue;
                    const int off = ks == 1 ? (pl == 0 ? aoff[grp][1] : aoff2[grp]) : pl * PLS + aoff[grp][0];
                    af[pl][grp] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(pb + off));
                }
#pragma unroll
            for (int r3 = 0; r3 < 3; ++r3) {
                const int rr = 2 - r3;
                const bf16x8 b = bw[rr * KS + ks];
#pragma unroll
                for (int pl = 0; pl < 3; ++pl)
#pragma unroll
                    for (int grp = 0; grp < NG; ++grp) {
                        if (pl >= np) continue;
                        const floatx4 c = (rr == 0 && ks == 0 && pl == 0) ? floatx4{0.f, 0.f, 0.f, 0.f}
                                                                         : acc[SL[rr]][grp][0];
                        acc[SL[rr]][grp][0] = TR ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, af[pl][grp], c, 0, 0, 0)
                                                 : __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[pl][grp], b, c, 0, 0, 0);
                    }
            }
        }
    };
    auto zero_slot = [&](auto S_) __attribute__((always_inline)) {
        constexpr int SR = decltype(S_)::value;
#pragma unroll
        for (int grp = 0; grp < NG; ++grp) acc[(SR + 1) % 3][grp][0] = floatx4{0.f, 0.f, 0.f, 0.f};
    };
    floatx4 pend[NG];
#pragma unroll
    for (int grp = 0; grp < NG; ++grp) pend[grp] = floatx4{0.f, 0.f, 0.f, 0.f};

    // ---- B, step j: epilogue 1 of intermediate row j - 3 (pend) into ring slot YW, the split of x row
    // j, conv 1 on it (intermediate row j - 2 completes into pend)
    auto stepB = [&](auto S_, int j) __attribute__((always_inline)) {
        constexpr int S6 = decltype(S_)::value;
        constexpr int S = S6 % 3;
        constexpr int D = (S + 2) % 3;
        constexpr int YW = (S6 + 1) & 1;
        const int RS = (6 % PD == 0) ? S6 % PD : j % PD;
        rows_wait<VMW_B>();  // this wave's part of x row j has landed
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        load_x((6 % PD == 0) ? (S6 + PD - 1) % PD : (j - 1 + PD) % PD, j - 1 + PD);
        uint32_t bx[8], hx;
        {
            const unsigned char* rw = raw + RS * rawslot;
#pragma unroll
            for (int e = 0; e < 8; ++e) bx[e] = *reinterpret_cast<const uint32_t*>(rw + rdx0 + e * RPB);
            hx = *reinterpret_cast<const uint32_t*>(rw + rdx_h);
        }
        {
            const int i1 = j - 3;
            const int r1 = p0 - 1 + i1;
            const bool irow = i1 >= 0 && i1 < n1 && r1 >= 0 && r1 < a.H;
            const int p = lane & 15, g = lane >> 4;
            unsigned char* yw = yr + YW * yslot;
#pragma unroll
            for (int grp = 0; grp < NG; ++grp) {
                const int q = q0 + 16 * grp + p;
                const bool okq = irow && q < a.W;
                uint32_t b4[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    float t;
                    if constexpr (E == 0) {
                        t = pend[grp][e] * scale + 0.0f;
                    } else if constexpr (E == 2) {
                        t = pend[grp][e] * es[e] + eb[e];
                        t = t < 0.0f ? 0.0f : t;
                    } else {
                        t = epi_act((pend[grp][e] * scale + bk[e]) * es[e] + eb[e], a.act1);
                    }
                    b4[e] = okq ? __float_as_uint(t) : 0u;
                }
                uint2 h2, m2, l2;
                split4p<false>(b4, h2, m2, l2);
                const int wo = yoct<CC>(q + 1, g >> 1) + 8 * (g & 1);
                *reinterpret_cast<uint2*>(yw + wo) = h2;
                *reinterpret_cast<uint2*>(yw + YPL + wo) = m2;
                *reinterpret_cast<uint2*>(yw + 2 * YPL + wo) = l2;
            }
        }
        {
            uint4 hi, mid, lo;
            split3<false>(bx, hi, mid, lo);
            *reinterpret_cast<uint4*>(slab + wa_i) = hi;
            *reinterpret_cast<uint4*>(slab + PL + wa_i) = mid;
            *reinterpret_cast<uint4*>(slab + 2 * PL + wa_i) = lo;
            uint16_t h16, m16, l16;
            split1(h_ok ? hx : 0u, h16, m16, l16);
            *reinterpret_cast<uint16_t*>(slab + wa_h) = h16;
            *reinterpret_cast<uint16_t*>(slab + PL + wa_h) = m16;
            *reinterpret_cast<uint16_t*>(slab + 2 * PL + wa_h) = l16;
        }
        {
            const int h = p0 - 2 + j;  // rows outside the image are zeros: their MFMAs add exact zeros
            if (j < nx && h >= 0 && h < a.H)
                mfmas(std::integral_constant<int, S>{}, std::true_type{}, slab);
            else
                zero_slot(std::integral_constant<int, S>{});
        }
#pragma unroll
        for (int grp = 0; grp < NG; ++grp) pend[grp] = acc[D][grp][0];
    };

    // ---- A, step j: conv 2 on intermediate row j - 4 (ring slot YR), epilogue 2 of output row j - 6
    // with conv_pair's whole-line DPP stores
    auto stepA = [&](auto S_, int j) __attribute__((always_inline)) {
        constexpr int S6 = decltype(S_)::value;
        constexpr int S = S6 % 3;
        constexpr int D = (S + 2) % 3;
        constexpr int YR = S6 & 1;
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        {
            const int i2 = j - 4, r2 = p0 - 1 + i2;
            if (i2 >= 0 && i2 < n1 && r2 >= 0 && r2 < a.H)
                mfmas(std::integral_constant<int, S>{}, std::false_type{}, yr + YR * yslot);
            else
                zero_slot(std::integral_constant<int, S>{});
        }
        const int o = j - 6;
        const bool orow = o >= 0 && o < rbe;
        const int g = lane >> 4;
        floatx4 vv[NG];
#pragma unroll
        for (int grp = 0; grp < NG; ++grp) {
            floatx4 v;
#pragma unroll
            for (int e = 0; e < 4; ++e)
                v[e] = E == 0 ? acc[D][grp][0][e] * scale + 0.0f
                       : E == 2 ? acc[D][grp][0][e] * es[0] + eb[0]
                                : (acc[D][grp][0][e] * scale + bk[0]) * es[0] + eb[0];
            if constexpr (E == 2) {
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = v[e] < 0.0f ? 0.0f : v[e];
            } else if constexpr (E != 0) {
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = epi_act(v[e], a.act2);
            }
            vv[grp] = v;
        }
        const bool hi8 = (lane & 8) != 0;
        floatx4 sa, sb;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            sa[e] = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(vv[0][e]), __float_as_int(vv[NG - 1][e]),
                                                               0x128, 0xf, 0xc, false));
            sb[e] = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(vv[NG - 1][e]), __float_as_int(vv[0][e]),
                                                               0x128, 0xf, 0x3, false));
        }
        const int q = q0 + (hi8 ? 16 : 0) + 4 * g;
        const uint32_t rowoff = (uint32_t)(orow ? p0 + o : 0) * a.W + (uint32_t)q;
        const uint32_t ca = (uint32_t)(lane & 7), cb = 8u + (uint32_t)(lane & 7);
        const bool ok = orow && q < a.W;
        rows_store<(NTS & 1) != 0>(ry, ok ? (ca * (uint32_t)HW + rowoff) * 4u : 0x7fffffffu, sa);
        rows_store<(NTS & 1) != 0>(ry, ok ? (cb * (uint32_t)HW + rowoff) * 4u : 0x7fffffffu, sb);
    };

    if (!roleA) {
#pragma unroll
        for (int r = 0; r < PD - 1; ++r) load_x(r, r);
    }
    {
        unsigned* red = reinterpret_cast<unsigned*>(yr);
        unsigned* thr = red + 16;
        uint4* fr = reinterpret_cast<uint4*>(yr + 4096);
        static_assert(4096 + 2 * NF * 64 * 16 <= 2 * yslot, "fragment scratch");
        bool fin1, fin2;
        const float scale1 = wq_prologue(a.q1, thr, red, 2 * NWR, fin1);
        wq_pack_rows_lds<CC>(a.q1, CC, CC, NT, KS, scale1, fin1, thr, fr, NF, true);
        const float scale2 = wq_prologue(a.q2, thr, red, 2 * NWR, fin2);
        wq_pack_rows_lds<CC>(a.q2, CC, CC, NT, KS, scale2, fin2, thr, fr + NF * 64, NF, true);
        const uint4* frw = fr + (roleA ? NF * 64 : 0);
#pragma unroll
        for (int f = 0; f < NF; ++f) bw[f] = __builtin_bit_cast(bf16x8, frw[f * 64 + lane]);
        scale = roleA ? scale2 : scale1;
        fin = roleA ? fin2 : fin1;
        if constexpr (E != 0) {
            const float *b = roleA ? a.b2 : a.b1, *ps = roleA ? a.ps2 : a.ps1, *pb = roleA ? a.pb2 : a.pb1;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int k = roleA ? (lane & 15) : 4 * (lane >> 4) + e;
                bk[e] = b ? b[k] : 0.0f;
                es[e] = ps ? ps[k] : 1.0f;
                eb[e] = pb ? pb[k] : 0.0f;
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if constexpr (E != 0) {
#pragma unroll
            for (int c = 0; c < 4; ++c) asm volatile("" : "+v"(bk[c]), "+v"(es[c]), "+v"(eb[c]));
        }
#pragma unroll
        for (int f = 0; f < NF; ++f) asm volatile("" : "+v"(bw[f]));
        if constexpr (E == 2) {
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                eb[c] = bk[c] * es[c] + eb[c];
                es[c] = scale * es[c];
            }
        }
        __syncthreads();  // scratch reads done: zero the intermediate planes and the x planes' zero slots
        for (int e = tid; e < (2 * yslot) / 16; e += blockDim.x)
            reinterpret_cast<uint4*>(yr)[e] = make_uint4(0u, 0u, 0u, 0u);
        if (lane < 3 && !roleA) *reinterpret_cast<uint4*>(slab + lane * PL + zero_off) = make_uint4(0u, 0u, 0u, 0u);
    }
    (void)fin;
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
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

static size_t pair_lds(int C, int waves, int pd, bool res, bool mw = false) {  // res: the compute waves' residual slots
    const int sw = 512 / C, wp = sw * waves;
    const int plane = (sw + 2) * 2 * C + 32;
    const int nf = 3 * (C == 16 ? 2 : 3) * (C / 16);
    const size_t slot = (mw && C == 16) ? ((size_t)C * (wp * 4 + 16) + 1023) / 1024 * 1024 : (size_t)C * wp * 4;
    return (size_t)pd * slot + 2 * 3 * (size_t)(7 * sw + 3) * 2 * C + (size_t)waves * 3 * plane +
           (res ? (size_t)waves * pd * kQResSlot : 0) + (C == 32 ? (size_t)nf * 64 * 16 : 0);
}

// One block per CU (7 waves); segments of RB output rows: the fewest segments that still
// give every CU a block, each recomputing 2 intermediate rows of its neighbours.
static bool pair_plan(PairPlan& pp, int N, int C, int H, int W, bool res, int pd, int nts, bool mw = false) {
    if (N <= 0 || H <= 0 || W <= 0 || W % 4 != 0 || (C != 16 && C != 32)) return false;
    const int sw = 512 / C;
    const int waves = (W + sw - 1) / sw;
    if (waves > 7) return false;
    if ((int64_t)C * H * W * 4 >= (1LL << 31)) return false;
    pp.C = C;
    pp.waves = waves;
    pp.pd = pd;
    pp.nts = nts;
    pp.lds = pair_lds(C, waves, pd, res, mw);
    if (pp.lds > 160 * 1024) return false;
    int nseg = std::max(1, (256 + N - 1) / N);
    nseg = std::min(nseg, std::max(1, H / 8));
    pp.RB = (H + nseg - 1) / nseg;
    pp.nseg = (H + pp.RB - 1) / pp.RB;
    const int64_t items = (int64_t)N * pp.nseg;
    if (items > INT_MAX / 2) return false;
    pp.blocks = (items + 7) / 8 * 8;
    return true;
}

template <int CC, int PD, int NTS>
static hipError_t launch_pair_t(const PairPlan& pp, const PairArgs& a, const float* x, float* y, bool res,
                                hipStream_t s) {
    const bool plain = !res && !a.b1 && !a.b2 && !a.ps1 && !a.pb1 && !a.ps2 && !a.pb2 && a.act1 == 0 && a.act2 == 0;
    const dim3 grid((unsigned)pp.blocks), block(64 * pp.waves);
#ifdef PO2Q_PAIR_STAMPS
    if (plain && getenv("PO2Q_STAMPS")) {
        PairArgs as = a;
        const size_t nst = (size_t)pp.blocks * 8 * 9;
        if (hipMalloc(&as.stamps, nst * 4) == hipSuccess) {
            (void)hipMemsetAsync(as.stamps, 0, nst * 4, s);
            hipLaunchKernelGGL((conv_pair<CC, PD, NTS, false, 0>), grid, block, pp.lds, s, x, y, as);
            std::vector<unsigned> h(nst);
            (void)hipStreamSynchronize(s);
            (void)hipMemcpy(h.data(), as.stamps, nst * 4, hipMemcpyDeviceToHost);
            (void)hipFree(as.stamps);
            double sum[9] = {0};
            for (size_t i = 0; i < nst; ++i) sum[i % 9] += h[i];
            const double waves = (double)pp.blocks * pp.waves, steps = sum[8] / waves;
            static const char* names[8] = {"top->wait", "vmcnt-wait", "barrier", "conv2-mfma", "epi2",
                                           "split-x", "conv1-mfma", "epi1"};
            double tot = 0;
            for (int i = 0; i < 8; ++i) tot += sum[i];
            fprintf(stderr, "[po2q stamps] C=%d blocks=%lld waves/block=%d steps/wave=%.1f cycles/step/wave=%.0f\n", CC,
                    (long long)pp.blocks, pp.waves, steps, tot / waves / steps);
            for (int i = 0; i < 8; ++i)
                fprintf(stderr, "  %-11s %8.0f cyc/step  %5.1f%%\n", names[i], sum[i] / waves / steps, 100.0 * sum[i] / tot);
            return hipGetLastError();
        }
    }
#endif
    if constexpr (PD >= 3 && (NTS == 3 || NTS == 1)) {
        if (a.mw && pp.waves == 7) {  // the memory-wave kernel: 7 compute waves + 1
            const dim3 block8(64 * 8);
            if (res) {  // residual == x, read from the ring (checked by the caller)
                if constexpr (PD >= 6) {
                    if (a.act1 == 1 && a.act2 == 1)
                        hipLaunchKernelGGL((conv_pair<CC, PD, NTS, true, 2, 0, 1>), grid, block8, pp.lds, s, x, y, a);
                    else
                        hipLaunchKernelGGL((conv_pair<CC, PD, NTS, true, 1, 0, 1>), grid, block8, pp.lds, s, x, y, a);
                    return hipGetLastError();
                }
                return hipErrorInvalidValue;
            }
            if (plain)
                hipLaunchKernelGGL((conv_pair<CC, PD, NTS, false, 0, 0, 1>), grid, block8, pp.lds, s, x, y, a);
            else
                hipLaunchKernelGGL((conv_pair<CC, PD, NTS, false, 1, 0, 1>), grid, block8, pp.lds, s, x, y, a);
            return hipGetLastError();
        }
    }
    if (plain)
        hipLaunchKernelGGL((conv_pair<CC, PD, NTS, false, 0>), grid, block, pp.lds, s, x, y, a);
    else if (res && a.act1 == 1 && a.act2 == 1)  // the BasicBlock form (resnet.py:55-71): ReLU / ReLU
        hipLaunchKernelGGL((conv_pair<CC, PD, NTS, true, 2>), grid, block, pp.lds, s, x, y, a);
    else if (res)
        hipLaunchKernelGGL((conv_pair<CC, PD, NTS, true, 1>), grid, block, pp.lds, s, x, y, a);
    else
        hipLaunchKernelGGL((conv_pair<CC, PD, NTS, false, 1>), grid, block, pp.lds, s, x, y, a);
    return hipGetLastError();
}

template <int PD>
static hipError_t launch_pair_rs(const PairPlan& pp, const PairArgs& a, const float* x, float* y, hipStream_t s) {
    const bool plain = !a.b1 && !a.b2 && !a.ps1 && !a.pb1 && !a.ps2 && !a.pb2 && a.act1 == 0 && a.act2 == 0;
    const dim3 grid((unsigned)pp.blocks), block(64 * 14);
    if (plain)
        hipLaunchKernelGGL((conv_pair_rs16<PD, 3, 0>), grid, block, pp.lds, s, x, y, a);
    else
        hipLaunchKernelGGL((conv_pair_rs16<PD, 3, 1>), grid, block, pp.lds, s, x, y, a);
    return hipGetLastError();
}

static hipError_t launch_pair(const PairPlan& pp, const PairArgs& a, const float* x, float* y, bool res,
                              hipStream_t s) {
    if (a.mw == 3) {  // RS: the role-split stage-1 pair (no residual; checked by the caller)
        if (res || pp.C != 16 || pp.waves != 7) return hipErrorInvalidValue;
        return pp.pd == 3 ? launch_pair_rs<3>(pp, a, x, y, s) : hipErrorInvalidValue;
    }
#ifdef PO2Q_PAIR_DIAG
    if (const char* dv = getenv("PO2Q_PAIR_DEBUG")) {
        const int dbg = atoi(dv);
        const dim3 grid((unsigned)pp.blocks), block(64 * pp.waves);
#define PO2Q_PD(v) \
        if (dbg == v && pp.C == 16 && pp.pd == 2 && pp.nts == 3 && !res) { \
            hipLaunchKernelGGL((conv_pair<16, 2, 3, false, 0, v>), grid, block, pp.lds, s, x, y, a); \
            return hipGetLastError(); \
        }
        PO2Q_PD(1) PO2Q_PD(2) PO2Q_PD(3) PO2Q_PD(4) PO2Q_PD(8) PO2Q_PD(12) PO2Q_PD(16) PO2Q_PD(19)
        PO2Q_PD(15) PO2Q_PD(31)
#undef PO2Q_PD
    }
#endif
#define PO2Q_PR(c, d, nt) \
    if (pp.C == c && pp.pd == d && pp.nts == nt) return launch_pair_t<c, d, nt>(pp, a, x, y, res, s);
#ifdef PO2Q_PAIR_ISA_ONLY  // ISA inspection builds (hipcc -S): the two default plans only
    PO2Q_PR(16, 5, 3) PO2Q_PR(32, 2, 3)
    return hipErrorInvalidValue;
#endif
    PO2Q_PR(16, 2, 0) PO2Q_PR(16, 2, 1) PO2Q_PR(16, 2, 3) PO2Q_PR(32, 2, 0) PO2Q_PR(32, 2, 3)
    PO2Q_PR(16, 5, 3) PO2Q_PR(16, 6, 3)
#undef PO2Q_PR
    return hipErrorInvalidValue;
}

}  // namespace po2q

// ------------------------------------------------------------------ C ABI --
namespace {

// variant knob: PO2Q_PAIR_VARIANT = prio * 100 + 20 + nts (prio 1: waves 4.. at issue priority 1;
// nts 3: non-temporal x loads and stores, 0: neither); default 23: 0.485 vs 0.508 ms at C = 16 and 0.353
// vs 0.364 at C = 32 (bs = 256, profiles/r02_pair_nt.log).  The measured-off ring depth 3 and the
// one-sided NT forms are gone, except 21 (non-temporal stores only), the C = 16 residual form's default.
void pair_variant(int& pd, int& nts, int& prio, int64_t C) {
    pd = 2;
    nts = 3;
    // priority 1 for waves 4..: 0.494 vs 0.504 / 0.500 ms at C = 16 (both store modes), mixed at
    // C = 32 (profiles/r02_pair_prio.log)
    prio = C == 16 ? 1 : 0;
    if (const char* e = getenv("PO2Q_PAIR_VARIANT")) {
        const int v = atoi(e) % 1000;
        const int d = (v / 10) % 10, t = v % 10;
        prio = v >= 100 ? 1 : 0;  // + 100: priority 1 for waves 4.. (an explicit variant sets it)
        if (d == 2 && (t == 0 || t == 3 || (t == 1 && C == 16))) {
            pd = d;
            nts = t;
        }
    }
}

bool pair_args_ok(int64_t N, int64_t C, int64_t H, int64_t W, int bits, int fsr, int mode, int act1, int act2) {
    if (N <= 0 || H <= 0 || W <= 0) {
        po2q::set_error("po2q: pair: sizes must be positive");
        return false;
    }
    if (C != 16 && C != 32) {
        po2q::set_error("po2q: pair: 16 or 32 channels only (ResNet56 stages 1 and 2)");
        return false;
    }
    if (mode != PO2Q_MODE_PO2 && mode != PO2Q_MODE_PO2_PLUS) {
        po2q::set_error("po2q: pair: mode must be po2 or po2+");
        return false;
    }
    if (bits < 1 || bits > 16) {
        po2q::set_error("po2q: bits must be in [1, 16]");
        return false;
    }
    const long lo = (long)fsr - (1L << (bits - 1)), hi = (long)fsr - 1;
    if (lo < -126 || hi > 127) {
        po2q::set_error("po2q: pair: the exponent window leaves the bf16 range");
        return false;
    }
    if (act1 < 0 || act1 > 3 || act2 < 0 || act2 > 3) {
        po2q::set_error("po2q: unknown activation");
        return false;
    }
    if (W % 4 != 0 || W > 7 * (512 / C)) {
        po2q::set_error("po2q: pair: W must be a multiple of 4 and at most 7 x 512 / C (224 for C = 16, 112 for 32)");
        return false;
    }
    return true;
}

}  // namespace

int po2q_qconv2d_pair_supported(int64_t N, int64_t C, int64_t H, int64_t W, int bits, int fsr, int mode) {
    // below 4 waves per block a block is too narrow to hide its per-row latency: two
    // single-conv launches are faster there (ResNet56 @32: 2.6 vs 2.0 ms per forward)
    if ((C == 16 || C == 32) && W <= 3 * (512 / C)) return 0;
    // C = 32 (stage 2 @112): round 2 measured the pair slower inside the ResNet56 chain (0.418 ms
    // against 2 x 0.197 for the single-conv kernel, profiles/r02_v7_kernel_stats.csv); after the
    // round-3 instruction diet it is 0.339 ms alone and the chain with stage-2 pairs runs 24.0k
    // against 23.4k img/s, 4 of 4 interleaved rounds on one box (profiles/r03_ab_stage2_pairs_v2.jsonl),
    // so it is advised.  PO2Q_PAIR_C32=0 turns the advice off (A/B runs).
    if (C == 32) {
        const char* e = getenv("PO2Q_PAIR_C32");
        if (e && e[0] == '0') return 0;
    }
    po2q::PairPlan pp;
    int pd, nts, prio;
    pair_variant(pd, nts, prio, C);
    return pair_args_ok(N, C, H, W, bits, fsr, mode, 0, 0) &&
                   po2q::pair_plan(pp, (int)N, (int)C, (int)H, (int)W, true, pd, nts)
               ? 1
               : 0;
}

int po2q_qconv2d_pair_f32(const float* x, const float* w1, const float* w2, float* y, int64_t N, int64_t C,
                          int64_t H, int64_t W, int bits, int fsr, int mode, const float* bias1, const float* bias2,
                          const float* post_scale1, const float* post_shift1, int act1, const float* post_scale2,
                          const float* post_shift2, const float* residual, int act2, void* stream) {
    if (!pair_args_ok(N, C, H, W, bits, fsr, mode, act1, act2)) return PO2Q_ERR_INVALID;
    if (!x || !w1 || !w2 || !y) {
        po2q::set_error("po2q: null pointer");
        return PO2Q_ERR_INVALID;
    }
    if (residual == y || x == y) {
        po2q::set_error("po2q: pair: y must not alias x or the residual");
        return PO2Q_ERR_INVALID;
    }
    if (po2q::pairw_applicable(N, C, H, W)) {  // stage 2 @112: 4 waves x 32 columns (po2q_conv_pairw.hip)
        const hipError_t e = po2q::pairw_launch(x, w1, w2, y, N, H, W, bits, fsr, mode, bias1, bias2, post_scale1,
                                                post_shift1, act1, post_scale2, post_shift2, residual, act2,
                                                reinterpret_cast<hipStream_t>(stream));
        if (e != hipSuccess) {
            po2q::set_error(std::string("po2q: pair launch: ") + hipGetErrorString(e));
            return PO2Q_ERR_HIP;
        }
        return PO2Q_OK;
    }
    po2q::PairPlan pp;
    int pd, nts, prio;
    pair_variant(pd, nts, prio, C);
    if (residual && C == 16 && !getenv("PO2Q_PAIR_VARIANT")) {
        // the BasicBlock form re-reads x as the residual five steps after its row DMA: with
        // temporal x loads that read hits L2, with non-temporal ones it goes back to memory.
        // Variant 21 (temporal x loads, non-temporal stores, no priority): 0.514 vs 0.551 ms,
        // 3 of 3 interleaved rounds (profiles/r03_ab_pair_res_temporal_x.jsonl)
        pd = 2;
        nts = 1;
        prio = 0;
    }
    if (!po2q::pair_plan(pp, (int)N, (int)C, (int)H, (int)W, residual != nullptr, pd, nts)) {
        po2q::set_error("po2q: pair: no plan for this shape");
        return PO2Q_ERR_UNSUPPORTED;
    }
    po2q::PairArgs a;
    a.N = (int)N; a.H = (int)H; a.W = (int)W;
    a.Wp = (512 / (int)C) * pp.waves;
    a.YPL = (7 * (512 / (int)C) + 3) * 2 * (int)C;  // the kernel's compile-time plane pitch
    a.RB = pp.RB; a.nseg = pp.nseg; a.items = (int)(N * pp.nseg);
    a.remap = (pp.blocks % 8 == 0) ? 1 : 0;
    const int lo = fsr - (1 << (bits - 1)), hi = fsr - 1;
    a.q1.w = w1; a.q1.n = (int)(C * C * 9); a.q1.lo = lo; a.q1.hi = hi; a.q1.mode = mode - 1;
    a.q2 = a.q1;
    a.q2.w = w2;
    a.b1 = bias1; a.b2 = bias2;
    a.ps1 = post_scale1; a.pb1 = post_shift1; a.act1 = act1;
    a.ps2 = post_scale2; a.pb2 = post_shift2; a.act2 = act2;
    a.res = residual;
    a.prio = prio;
    a.stamps = nullptr;
    // The memory-wave kernel with a PD-slot x ring: the default at C = 16 (PD 5; 6 for the identity
    // residual read from the ring): 0.4286 vs 0.4385 ms for the plain pair 16 @224 bs 256, 4
    // interleaved rounds (profiles/r04_pair_mw_ab.jsonl); at C = 32 no gain (0.3401 vs 0.3394), and
    // ring depths 3, 4 and 6 for the plain pair no different (r04_pair_mw_ab.jsonl): those variants are
    // gone.  PO2Q_PAIR_MW=0 selects the one-role kernel (A/B and test knob).
    a.mw = 0;
    // The role-split stage-1 pair (conv_pair_rs16, 3 x-ring slots) for the forms without a residual at
    // seven strips: 0.392 vs 0.414 ms for the memory-wave kernel, bench 25.83k vs 25.43k img/s
    // (profiles/r06_pair16_rs_ab.jsonl; ring depths 2 / 4: 0.392 / 0.398).  PO2Q_PAIR_RS=0 turns it off;
    // an explicit PO2Q_PAIR_MW or PO2Q_PAIR_VARIANT selects the kernels those knobs name (A/B and tests).
    {
        const char* rsv = getenv("PO2Q_PAIR_RS");
        const bool rs_on = rsv ? rsv[0] != '0' : (!getenv("PO2Q_PAIR_MW") && !getenv("PO2Q_PAIR_VARIANT"));
        const int d = 3;
        if (rs_on && C == 16 && W > 6 * 32 && !residual) {
            a.mw = 3;
            if (!po2q::pair_plan(pp, (int)N, (int)C, (int)H, (int)W, false, d, 3)) {
                po2q::set_error("po2q: pair: no role-split plan for this shape");
                return PO2Q_ERR_UNSUPPORTED;
            }
            const hipError_t e = po2q::launch_pair(pp, a, x, y, false, reinterpret_cast<hipStream_t>(stream));
            if (e != hipSuccess) {
                po2q::set_error(std::string("po2q: pair launch: ") + hipGetErrorString(e));
                return PO2Q_ERR_HIP;
            }
            return PO2Q_OK;
        }
    }
    const char* mv = getenv("PO2Q_PAIR_MW");
    if (!mv && C == 16 && !getenv("PO2Q_PAIR_VARIANT")) mv = "5";
    if (mv) {
        const int d = atoi(mv);
        // with a residual: only the identity shortcut (residual == x), from a 6-slot ring
        const bool ring_res = residual != nullptr && residual == x && C == 16;
        const bool seven = W > 6 * (512 / C);  // the memory-wave kernel exists for 7 compute waves only
        if (d == 5 && C == 16 && seven && (!residual || ring_res)) {
            a.mw = 1;
            pd = residual ? 6 : d;
            nts = 3;  // with the ring residual no x row is re-read from memory: non-temporal loads
            if (!po2q::pair_plan(pp, (int)N, (int)C, (int)H, (int)W, false, pd, nts, true)) {
                po2q::set_error("po2q: pair: no memory-wave plan for this shape");
                return PO2Q_ERR_UNSUPPORTED;
            }
        }
    }
    const hipError_t e = po2q::launch_pair(pp, a, x, y, residual != nullptr, reinterpret_cast<hipStream_t>(stream));
    if (e != hipSuccess) {
        po2q::set_error(std::string("po2q: pair launch: ") + hipGetErrorString(e));
        return PO2Q_ERR_HIP;
    }
    return PO2Q_OK;
}
