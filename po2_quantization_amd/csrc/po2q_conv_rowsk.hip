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
#include "po2q_quant_dev.h"
#include "po2q_rows_dev.h"
#include "po2q_x3_dev.h"

namespace po2q {

namespace {

constexpr int kKSW = 32;                       // strip width (2 pixel groups of 16)
constexpr int kKWC = kKSW + 2;                 // halo columns
template <int C> constexpr int kKPlane = kKWC * C * 2;          // bytes per bf16 plane
template <int C> constexpr int kKRawInt = C * kKSW * 4;        // raw interior [C][32] fp32
template <int C> constexpr int kKRawSlot = kKRawInt<C> + 4 * 256;  // + 4 waves x 64 halo dwords
template <int C> constexpr int kKTile = C * kKSW * 4;           // output row tile [K][32] fp32
template <int C, int PD, bool TT>
constexpr int kKLds = 2 * 3 * kKPlane<C> + PD * kKRawSlot<C> + (TT ? 2 * kKTile<C> : 0);

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
    const float* res;  // RES: y = act(y * ps + pb + res), res [N, K, P, Q] (loader wave DMAs it)
    WQuant q;          // FP: raw weights + quantizer parameters
};

// The LW loader wave: every DMA of the block, the layout the MFMA waves' own DMAs
// would have produced (interior: instruction i, lane l -> channel 8i + (l >> 3),
// columns 4(l & 7) .. +3 at raw[c][col]; halo: lane l -> side l / C, channel l % C).
// Row j is published by the barrier of step j - 1 (barrier -1: the preamble's), and
// its slot is refilled with row j + PD after the barrier of step j, so it executes
// exactly the MFMA waves' barriers: one preamble, one per (whole-triple) step and the
// TT flush.
template <int C, int PD, bool TT, bool RES, bool NTL>
__device__ __forceinline__ void loader_wave(const float* __restrict__ x, const RowsKArgs& a, unsigned char* raw,
                                            unsigned char* resb, int n, int q0, int p0, int nrows, int rbe) {
    constexpr int NI = C / 8 + 1;  // instructions per row: C/8 interior + 1 halo
    static_assert(2 * C <= 64, "one halo instruction per row");
    const int lane = threadIdx.x & 63;
    const int HW = a.H * a.W;
    const uint32_t cstride = (uint32_t)HW * 4u;
    const __amdgpu_buffer_rsrc_t rs = rows_rsrc(x + (int64_t)n * C * HW, C * HW * 4);
    const int gq4 = q0 + 4 * (lane & 7);
    const bool qi_ok = gq4 < a.W;
    const uint32_t vi0 = (uint32_t)(lane >> 3) * cstride + (uint32_t)gq4 * 4u;
    const int hside = lane / C, hch = lane % C;
    const int gqh = hside ? q0 + kKSW : q0 - 1;
    const bool qh_ok = gqh >= 0 && gqh < a.W;
    const uint32_t vh0 = (uint32_t)hch * cstride + (uint32_t)gqh * 4u;
    const uint32_t raw_lds = (uint32_t)(uintptr_t)raw;
    // RES: the residual row stored in step js (output row p0 + js - 3) into slot js & 1,
    // [K][32 columns] like the output tile (unswizzled): 8 channels x 128 B per instruction
    const int PQ = a.P * a.Q;
    const __amdgpu_buffer_rsrc_t rr = rows_rsrc(RES ? a.res + (int64_t)n * C * PQ : x, RES ? C * PQ * 4 : 4);
    const uint32_t vr0 = (uint32_t)(lane >> 3) * (uint32_t)PQ * 4u + (uint32_t)gq4 * 4u;
    auto lres = [&](int js) __attribute__((always_inline)) {
        const int orow = js - 3;
        const bool ok = orow >= 0 && orow < rbe && gq4 < a.Q;
        const uint32_t vo = ok ? vr0 + (uint32_t)(p0 + orow) * (uint32_t)a.Q * 4u : 0x7fffffffu;
        const uint32_t base = (uint32_t)(uintptr_t)resb + (uint32_t)((js & 1) * kKTile<C>);
#pragma unroll
        for (int i = 0; i < C / 8; ++i) rows_dma16(rr, vo, i * 8u * (uint32_t)PQ * 4u, base + (uint32_t)i * 1024u);
    };
    auto lrow = [&](int sl, int j) __attribute__((always_inline)) {
        const int h = p0 - 1 + j;
        const bool hok = j < nrows && h >= 0 && h < a.H;
        const uint32_t roff = (uint32_t)(hok ? h : 0) * (uint32_t)a.W * 4u;
        const uint32_t vo = (hok && qi_ok) ? vi0 + roff : 0x7fffffffu;
        const uint32_t base = raw_lds + (uint32_t)(sl * kKRawSlot<C>);
#pragma unroll
        for (int i = 0; i < C / 8; ++i) rows_dma16<NTL>(rs, vo, i * 8u * cstride, base + (uint32_t)i * 1024u);
        rows_dma4<NTL>(rs, (hok && qh_ok) ? vh0 + roff : 0x7fffffffu, base + (uint32_t)kKRawInt<C>);
    };
#pragma unroll
    for (int r = 0; r < PD; ++r) lrow(r, r);
    rows_wait<(PD - 1) * NI>();  // row 0
    __builtin_amdgcn_s_barrier();
    const int steps = (nrows + 2) / 3 * 3;  // the MFMA waves run whole triples of steps
    int sl = 0;
    for (int j = 0; j < steps; ++j) {
        rows_wait<(PD - 2) * NI>();  // row j + 1 (issued after it: rows j + 2 .. j + PD - 1)
        __builtin_amdgcn_s_barrier();
        if constexpr (RES) lres(j + 1);  // older than the row DMA below: the next wait covers it
        lrow(sl, j + PD);  // the slot of row j, split before this barrier
        sl = sl + 1 == PD ? 0 : sl + 1;
    }
    if (TT && nrows % 3 == 0) {
        if constexpr (RES) rows_wait<0>();  // the flushed row's residual
        __builtin_amdgcn_s_barrier();
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// PD: halo rows in flight per wave (raw ring slots): 2 or 3 (a divisor of the 6-step
//     unroll)
// TT: output rows leave through a double-buffered LDS tile [K][32 columns]: a row
//     completed in step j is stored in step j+1 as 128-byte channel runs (8 channels
//     per wave instruction) instead of one 64-byte run per channel and column group
// LW: a fifth, loader wave issues every DMA of the block (and joins the per-row
//     barrier); the four MFMA waves issue no global loads, only stores.  A wave's
//     loads queue behind its own earlier stores, so a wave that both streams stores
//     and loads gets about half the store rate of a store-only wave (r01_v13 ablation)
// DBG (diagnostic builds only, -DPO2Q_ROWS_DIAG; timing only, outputs wrong): bit 1 =
// halo-column DMAs read nothing, 2 = no MFMAs, 4 = no split, 8 = interior DMAs read
// nothing, 16 = stores write nothing (dropped instructions still issue and count),
// 32 = TT stores non-temporal, 64 = no wait for the DMAs (vmcnt 31), 128 = no DMA
// instructions in the loop, 256 = no TT tile LDS traffic.
// Product builds: DBG = 0.
// NTS (plan field nts, autotune candidates): bit 0 = output stores, bit 1 = x loads with
// the non-temporal policy
// RES (with TT, EPI): the residual add inside the kernel (the loader wave -- or, without
//     LW, each MFMA wave for the channels its tile stores cover -- DMAs the residual rows
//     into a 2-slot ring next to the output tile; act after the add)
// FP (plan field fp, not with LW): the block reduces max|w| and each wave quantizes +
//     packs its own VGPR-resident B fragments (po2q_quant_dev.h wq_*): one launch per layer
// PIPE (not with LW / RES / FP): the split runs one row ahead.  Step j's MFMAs read the planes of
//     row j (split in step j - 1) while the wave splits row j + 1 into the other plane buffer,
//     between its first k-step's MFMAs and the next fragment reads, and the step's one barrier
//     moves to its end: the split's vector and LDS work issues beside the matrix work instead of
//     in front of it, behind a barrier.  Same arithmetic, same outputs bit for bit.
template <int C, int PD, bool TT, bool LW, bool EPI = false, int DBG = 0, int NTS = 0, bool RES = false,
          bool FP = false, bool PIPE = false>
__global__ __launch_bounds__(LW ? kThreads + 64 : kThreads, C == 64 ? (TT ? 2 : 3) : 4) void conv_rowsk(const float* __restrict__ x, const uint4* __restrict__ wpk,
                                                          const float* __restrict__ scale_p,
                                                          const float* __restrict__ bias, float* __restrict__ y,
                                                          RowsKArgs a) {
    static_assert(!PIPE || (!LW && !RES && !FP && DBG == 0), "pipelined split: plain MFMA-wave plans");
    // FPF (-DPO2Q_ROWSK_FPF=1, TT plans only: 2 blocks per CU leave the VGPRs for the second
    // fragment set; the 3-block direct-store plans would spill): A fragments one k-step ahead.
    // Off: no measurable change at stage 3 (profiles/r04_rowsk_pipe_ab.jsonl, call r04_24)
#ifndef PO2Q_ROWSK_FPF
#define PO2Q_ROWSK_FPF 0
#endif
    constexpr bool FPF = PO2Q_ROWSK_FPF != 0 && TT;
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
    unsigned char* tile = raw + PD * kKRawSlot<C>;  // TT: 2 output row tiles
    unsigned char* resb = tile + 2 * kKTile<C>;     // RES: 2 residual row tiles

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

    if constexpr (LW) {
        if (wave == 4) {
            loader_wave<C, PD, TT, RES, (NTS & 2) != 0>(x, a, raw, resb, n, q0, p0, nrows, rbe);
            return;
        }
    }

    // ---- this wave's weights: B[r][ks = chunk*3 + s] for output channels 16w..16w+15
    static_assert(!(FP && LW), "the loader wave keeps its own barrier count");
    bf16x8 bw[3][KSC];
    float scale;
    if constexpr (FP) {
        // scratch in the raw ring, free until the first DMA below
        unsigned* red = reinterpret_cast<unsigned*>(raw);
        unsigned* thr = red + 16;
        bool fin;
        scale = wq_prologue(a.q, thr, red, 4, fin);
        // one tap row's fragments at a time, packed by the whole block from coalesced weight reads
        // into the (still unused) planes, then each wave takes its own (wq_pack_tap_row_lds)
        uint4* fr = reinterpret_cast<uint4*>(planes);
        static_assert(KSC * WN * 64 * 16 <= 2 * 3 * PL, "fragment scratch in the planes");
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            wq_pack_tap_row_lds<C>(a.q, C, 32, WN, KSC, r, scale, fin, thr, fr);
#pragma unroll
            for (int ks = 0; ks < KSC; ++ks) bw[r][ks] = __builtin_bit_cast(bf16x8, fr[(ks * WN + wn) * 64 + lane]);
            __syncthreads();  // every wave's reads of row r done before row r + 1 (or the splits) overwrite fr
        }
        // (the last barrier also orders every threshold read before the ring's DMAs)
    } else {
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int ks = 0; ks < KSC; ++ks)
                bw[r][ks] = __builtin_bit_cast(bf16x8, wpk[((r * KSC + ks) * WN + wn) * 64 + lane]);
        scale = *scale_p;
    }
    const int kout = 16 * wn + (lane & 15);
    float bk = bias ? bias[kout] : 0.0f;
    float eps_ = (EPI && a.ps) ? a.ps[kout] : 1.0f;
    float epb_ = (EPI && a.pb) ? a.pb[kout] : 0.0f;
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int ks = 0; ks < KSC; ++ks) asm volatile("s_waitcnt vmcnt(0)" : "+v"(bw[r][ks]));
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(bk), "+v"(eps_), "+v"(epb_));
    auto outv = [&](float accv) __attribute__((always_inline)) {
        const float v = accv * scale + bk;
        if constexpr (EPI && RES)
            return v * eps_ + epb_;  // the activation follows the residual add (store_tile)
        else if constexpr (EPI)
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

    auto load_row = [&](auto SL_, int j) __attribute__((always_inline)) {
        constexpr int sl = decltype(SL_)::value;
        const int h = p0 - 1 + j;
        const bool hok = j < nrows && h >= 0 && h < a.H;
        const uint32_t roff = (uint32_t)(hok ? h : 0) * (uint32_t)a.W * 4u;
        const uint32_t vo = (hok && qi_ok && !(DBG & 8)) ? vi0 + roff : 0x7fffffffu;
        const uint32_t voh = (hok && qh_ok && !(DBG & 1)) ? vh0 + roff : 0x7fffffffu;
        const uint32_t base = raw_lds + (uint32_t)(sl * RAWS);
#pragma unroll
        for (int i = 0; i < DPW; ++i) rows_dma16<(NTS & 2) != 0>(rs, vo, i * soff1, base + (uint32_t)(DPW * wave + i) * 1024u);
        rows_dma4<(NTS & 2) != 0>(rs, voh, base + (uint32_t)RAWI + (uint32_t)wave * 256u);
    };
    // RES without LW: per step this wave first DMAs the residual of the row its store_tile
    // writes in the NEXT step (NR instructions, the channels of that store), then the x row
    constexpr int NR = (RES && !LW) ? NGW : 0;
    static_assert(!RES || TT, "the residual rides on the TT output tile");
    // vm ops issued after a row's DMAs (step j-PD) until row j is split: that step's
    // stores, then per later step the residual and x DMAs of one more row and that step's stores
    constexpr int VMW = (PD - 1) * (NR + DPW + 1 + NGW) + NGW;
    // vm ops issued after the residual DMAs of step j-1 until step j's store_tile: step j-1's
    // x DMAs and stores, step j's residual and x DMAs
    constexpr int RW = 2 * (DPW + 1) + NGW + NR;
    const int PQ = a.P * a.Q;
    const __amdgpu_buffer_rsrc_t rres = rows_rsrc(NR ? a.res + (int64_t)n * K * PQ : x, NR ? K * PQ * 4 : 4);
    const uint32_t vr0 = (uint32_t)((K / 4) * wave + (lane >> 3)) * (uint32_t)PQ * 4u + (uint32_t)gq4 * 4u;
    // the residual row store_tile writes in step js (output row p0 + js - 3) into slot js & 1,
    // [K][32 columns] unswizzled: instruction i, lane l -> channel (K/4)w + 8i + (l >> 3)
    auto load_res = [&](int js) __attribute__((always_inline)) {
        if constexpr (NR != 0) {
            const int orow = js - 3;
            const bool ok = orow >= 0 && orow < rbe && gq4 < a.Q;
            const uint32_t vo = ok ? vr0 + (uint32_t)(p0 + orow) * (uint32_t)a.Q * 4u : 0x7fffffffu;
            const uint32_t base = (uint32_t)(uintptr_t)resb + (uint32_t)((js & 1) * kKTile<C>) +
                                  (uint32_t)((K / 4) * wave) * (kKSW * 4u);
#pragma unroll
            for (int i = 0; i < NR; ++i) rows_dma16(rres, vo, i * 8u * (uint32_t)PQ * 4u, base + (uint32_t)i * 1024u);
        }
    };
    const __amdgpu_buffer_rsrc_t ry = rows_rsrc(y + (int64_t)n * K * PQ, K * PQ * 4);

    // TT stores: wave w, instruction i: lane l -> channel (K/4)w + 8i + (l >> 3), columns
    // q0 + 4(l & 7) .. +3 (the tile's 16-byte blocks are XOR-swizzled by channel)
    auto store_tile = [&](const unsigned char* tr, int o, bool orow, int rslot) __attribute__((always_inline)) {
        const int sb = lane & 7;
        const int q = q0 + 4 * sb;
#pragma unroll
        for (int i = 0; i < NGW; ++i) {
            const int c = (K / 4) * wave + 8 * i + (lane >> 3);
            floatx4 v = floatx4{0.f, 0.f, 0.f, 0.f};
            if constexpr (!(DBG & 256)) v = *reinterpret_cast<const floatx4*>(tr + c * (kKSW * 4) + ((sb ^ (c & 7)) << 4));
            if constexpr (RES) {
                const floatx4 r = *reinterpret_cast<const floatx4*>(resb + rslot * kKTile<C> + c * (kKSW * 4) + 16 * sb);
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = epi_act(v[e] + r[e], a.act);
            }
            const uint32_t vo = (uint32_t)c * (uint32_t)PQ + (uint32_t)(orow ? o : 0) * a.Q + (uint32_t)q;
            rows_store<(NTS & 1) != 0 || (DBG & 32) != 0>(ry, (orow && q < a.Q && !(DBG & 16)) ? vo * 4u : 0x7fffffffu, v);
        }
    };

    // exact split of halo row rw (this wave's channels + halo values) into the planes at pb
    auto split_row = [&](const unsigned char* rw, unsigned char* pb) __attribute__((always_inline)) {
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
            // halo value hv = HPW * wave + lane: own DMA at [wave][lane], LW's at [hv]
            const int hoff = LW ? 4 * (HPW * wave + lane) : wave * 256 + 4 * lane;
            split1(*reinterpret_cast<const uint32_t*>(rw + RAWI + hoff), h16, m16, l16);
            *reinterpret_cast<uint16_t*>(pb + wa_h) = h16;
            *reinterpret_cast<uint16_t*>(pb + PL + wa_h) = m16;
            *reinterpret_cast<uint16_t*>(pb + 2 * PL + wa_h) = l16;
        }
    };

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
        [[maybe_unused]] const unsigned char* rw = raw + RS * RAWS;
        if constexpr (LW || PIPE) {
            // (LW: the loader published row j at the previous barrier; PIPE: row j was split in
            // step j - 1)
        } else if constexpr (DBG & 64) {
            rows_wait<31>();
        } else {
            rows_wait<VMW>();  // this wave's DMAs of row j have landed
        }
        if constexpr (!PIPE) {
            if constexpr (!(DBG & 4)) split_row(rw, pb);
            // publish the planes: LDS writes done, then the block barrier (no memory fence:
            // the prefetches and stores in flight must not be waited for)
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            // refill the raw slot this wave just split (its own data only)
            if constexpr (!(DBG & 128) && !LW) {
                load_res(j + 1);
                load_row(std::integral_constant<int, RS>{}, j + PD);
            }
        }
        // PIPE: end of step -- publish row j + 1's planes and this step's output tile, then refill
        // row j + 1's raw slot with row j + 1 + PD
        auto fin = [&]() __attribute__((always_inline)) {
            if constexpr (PIPE) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
                load_row(std::integral_constant<int, (S6 + 1) % PD>{}, j + 1 + PD);
            }
        };
        // MFMAs: halo row j feeds output halo-index j+1 (r=0), j (r=1), j-1 (r=2)
        constexpr int SL[3] = {(S + 1) % 3, S, (S + 2) % 3};
        // tap row rr of halo row j lands on segment output row j - rr: the edge steps (j < 2 or
        // j >= rbe) skip the MFMAs whose output lies outside the segment.  One wave-uniform
        // branch per step picks the guarded or the branch-free body: a test per tap row inside
        // the k-step loop split the MFMA stream into blocks the scheduler could not interleave
        // (26 branches and ~110 s_waitcnt per step in the loop's ISA).
        auto mma = [&](auto G_, auto&& after0) __attribute__((always_inline)) {
            constexpr bool G = decltype(G_)::value;
            // A fragments one k-step ahead (FPF): k-step ks + 1's reads are issued before k-step ks's
            // MFMAs, so their LDS latency runs under 3 x 3 x NGW MFMAs instead of stalling the first
            bf16x8 af[2][3][NGW];
            auto ldf = [&](bf16x8 (&f)[3][NGW], int ks) __attribute__((always_inline)) {
#pragma unroll
                for (int pl = 0; pl < 3; ++pl)
#pragma unroll
                    for (int grp = 0; grp < NGW; ++grp)
                        f[pl][grp] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(pb + pl * PL + aoff[grp][ks]));
            };
            if constexpr (FPF && !(DBG & 2)) ldf(af[0], 0);
#pragma unroll
            for (int ks = 0; ks < KSC && !(DBG & 2); ++ks) {
                bf16x8 (&cf)[3][NGW] = af[FPF ? (ks & 1) : 0];
                if constexpr (FPF) {
                    if (ks + 1 < KSC) ldf(af[(ks + 1) & 1], ks + 1);
                } else {
                    ldf(cf, ks);
                }
#pragma unroll
                for (int rr = 0; rr < 3; ++rr) {
                    if (G && (j - rr < 0 || j - rr >= rbe)) continue;
#pragma unroll
                    for (int pl = 0; pl < 3; ++pl)
#pragma unroll
                        for (int grp = 0; grp < NGW; ++grp)
                            acc[SL[rr]][grp] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cf[pl][grp], bw[rr][ks],
                                                                                      acc[SL[rr]][grp], 0, 0, 0);
                }
                if (ks == 0) after0();
            }
        };
        if constexpr (PIPE) {
            // row j + 1 (raw slot (S6 + 1) % PD) into the other plane buffer, beside k-step 0's MFMAs
            auto nxt = [&]() __attribute__((always_inline)) {
                rows_wait<(PD - 1) * (DPW + 1 + NGW)>();  // this wave's DMAs of row j + 1 have landed
                split_row(raw + ((S6 + 1) % PD) * RAWS, planes + (1 - B2) * 3 * PL);
            };
            if (j >= 2 && j < rbe)
                mma(std::false_type{}, nxt);
            else
                mma(std::true_type{}, nxt);
        } else {
            auto none = []() __attribute__((always_inline)) {};
            if (j >= 2 && j < rbe)
                mma(std::false_type{}, none);
            else
                mma(std::true_type{}, none);
        }
        // output halo-index j-1 (row p0 + j - 2) is complete
        constexpr int D = (S + 2) % 3;
        if constexpr (TT) {
            // store the row completed in the previous step (tile 1 - B2, published by
            // this step's barrier), then park this step's row in tile B2
            // (the loop runs whole triples of steps: steps past nrows - 1 only store)
            if constexpr (NR != 0) rows_wait<RW>();  // this row's residual (DMA'd in step j - 1)
            store_tile(tile + (1 - B2) * kKTile<C>, p0 + j - 3, j >= 3 && j - 3 < rbe, B2);
            unsigned char* tw = tile + B2 * kKTile<C>;
#pragma unroll
            for (int grp = 0; grp < NGW; ++grp) {
                floatx4 v;
                v[0] = outv(acc[D][grp][0]);
                v[1] = outv(acc[D][grp][1]);
                v[2] = outv(acc[D][grp][2]);
                v[3] = outv(acc[D][grp][3]);
                const int bi = 4 * (g0 + grp) + (lane >> 4);
                if constexpr (!(DBG & 256))
                    *reinterpret_cast<floatx4*>(tw + kout * (kKSW * 4) + ((bi ^ (kout & 7)) << 4)) = v;
                acc[D][grp] = floatx4{0.f, 0.f, 0.f, 0.f};
            }
            fin();
            return;
        }
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
            rows_store<(NTS & 1) != 0>(ry, (orow && q < a.Q && !(DBG & 16)) ? (yk + (uint32_t)q) * 4u : 0x7fffffffu, v);
            acc[D][grp] = floatx4{0.f, 0.f, 0.f, 0.f};
        }
        fin();
    };

    {
        const floatx4 z = floatx4{0.f, 0.f, 0.f, 0.f};
        auto pre = [&](auto R_) __attribute__((always_inline)) {
            load_res(decltype(R_)::value - PD + 1);  // no output row yet: counted, out of range
            load_row(R_, decltype(R_)::value);
#pragma unroll
            for (int i = 0; i < NGW; ++i) rows_store<(NTS & 1) != 0>(ry, 0x7fffffffu, z);
        };
        if constexpr (LW) {
            __builtin_amdgcn_s_barrier();  // the loader has rows 0 .. PD-1 in flight, row 0 landed
        } else {
            pre(std::integral_constant<int, 0>{});
            pre(std::integral_constant<int, 1>{});
            if constexpr (PD >= 3) pre(std::integral_constant<int, 2>{});
            if constexpr (PIPE) {
                rows_wait<VMW>();  // row 0
                split_row(raw, planes);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
                load_row(std::integral_constant<int, 0>{}, PD);
            }
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
    if (TT && nrows % 3 == 0) {
        // the last row (parked by step nrows - 1; with nrows % 3 != 0 the loop's extra
        // step nrows has stored it)
        if constexpr (NR != 0) rows_wait<0>();  // the flushed row's residual
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        store_tile(tile + ((nrows - 1) & 1) * kKTile<C>, p0 + rbe - 1, true, nrows & 1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // trailing DMAs land before the wave ends
}

// ------------------------------------------------------------------ planning --
// Candidates for 3x3 / s1 / p1 / C = K = 64 (plan kind bf16x3_rows with vrx = 1:
// output channels across the block's waves).  Weight pack: the row layout
// [r][ks = chunk*3 + s][nt][lane][8] (po2q_quant.hip, CC = 32, 2 chunks).
static int rowsk_lds(int C, int pd, bool tt) {
#define PO2Q_L(c, d) \
    if (C == c && pd == d) return tt ? kKLds<c, d, true> : kKLds<c, d, false>;
    PO2Q_L(64, 2) PO2Q_L(64, 3) PO2Q_L(32, 2) PO2Q_L(32, 3)
#undef PO2Q_L
    return 1 << 30;
}

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
    // vrx = 2: stores through the LDS output tile (TT); pd: prefetch depth (halo rows in
    // flight per wave)
    // vrx: 1 = direct stores, 2 = stores through the LDS output tile (TT), 3 = TT with
    // the loader wave (LW, C = 32); pd: rows in flight per wave
    const int vrxs[3] = {b.C == 64 ? 1 : 3, 2, b.C == 64 ? 0 : 1};
    for (int vrx : vrxs)
        for (int pd : {3, 2}) {
            if (vrx == 0 || (vrx == 3 && pd < 3)) continue;  // LW: two rows in flight at least
            ConvPlan c = p;
            c.pd = pd;
            c.vrx = vrx;
            const bool tt = vrx >= 2;
            c.lds_bytes = rowsk_lds(b.C, pd, tt);
            // blocks resident per chip: VGPR budget (C = 64: 3 per CU, 2 with TT; C = 32: 4)
            // and LDS (160 KiB per CU)
            const int per_cu = std::min(b.C == 64 ? (tt ? 2 : 3) : 4, (int)(163840 / c.lds_bytes));
            const int slots = 256 * per_cu;
            std::vector<std::pair<double, int>> rbs;
            for (int rb = 4; rb <= p.P; ++rb) {
                const int nseg = (p.P + rb - 1) / rb;
                if (rb != (p.P + nseg - 1) / nseg) continue;
                const int64_t items = (int64_t)p.N * nseg * p.tilesQ;
                if (items > INT_MAX / 2) continue;
                rbs.push_back({(double)((items + slots - 1) / slots) * (rb + 2), rb});
            }
            std::sort(rbs.begin(), rbs.end());
            for (int i = 0; i < (int)rbs.size() && i < 2; ++i) {
                ConvPlan d = c;
                d.TP = rbs[i].second;
                d.tilesP = (p.P + d.TP - 1) / d.TP;
                const int64_t items = (int64_t)p.N * d.tilesP * d.tilesQ;
                d.blocks = (items + 7) / 8 * 8;
                out.push_back({0.9 + 0.001 * i + (pd == 2 ? 0.01 : 0.0) + (vrx == vrxs[0] ? 0.0 : 0.02), d});
                // C = 64 direct stores with fused weight staging (one launch per layer): an autotune
                // candidate, not the heuristic default -- every block re-packs the 36,864 weights, so
                // even the cooperative staging leaves it at 0.298 ms against 0.164 ms + a ~7 us pack
                // for the packed plan at bs 256 @56 (profiles/r06_plan_sweep_fp.jsonl)
                if (b.C == 64 && vrx == 1) {
                    ConvPlan f = d;
                    f.fp = 1;
                    out.push_back({0.95 + 0.001 * i + (pd == 2 ? 0.01 : 0.0), f});
                }
                // the default variants (C = 64 direct stores, C = 32 loader wave) also with
                // non-temporal output stores (nts 1), non-temporal x loads (2) or both (3)
                if ((b.C == 64 && vrx == 1) || (b.C == 32 && vrx == 3))
                    for (int nts : {1, 2, 3}) {
                        d.nts = nts;
                        out.push_back({0.905 + 0.001 * i + 0.0001 * nts + (pd == 2 ? 0.01 : 0.0), d});
                    }
            }
        }
}

hipError_t launch_conv_rowsk(const ConvPlan& p, const float* x, const uint16_t* packed, const float* scale,
                             const float* bias, float* y, hipStream_t s, const float* ps, const float* pb,
                             int act, bool epi, const WQuant& q) {
    RowsKArgs a;
    a.N = p.N; a.H = p.H; a.W = p.W; a.P = p.P; a.Q = p.Q;
    a.RB = p.TP; a.nseg = p.tilesP; a.nstrip = p.tilesQ;
    a.items = p.N * p.tilesP * p.tilesQ;
    a.remap = (p.blocks % 8 == 0) ? 1 : 0;
    a.ps = ps;
    a.pb = pb;
    a.act = act;
    a.res = nullptr;
    a.q = q;
    if (p.fp) {  // fused weight staging: C = 64 direct-store plans
        if (!q.w || p.vrx != 1 || p.C != 64 || p.nts) return hipErrorInvalidValue;
#define PO2Q_RKF(d, e)                                                                                     \
    if (p.pd == d && epi == e) {                                                                             \
        hipLaunchKernelGGL((conv_rowsk<64, d, false, false, e, 0, 0, false, true>), dim3((unsigned)p.blocks), \
                           dim3(kThreads), p.lds_bytes, s, x, reinterpret_cast<const uint4*>(packed), scale, bias, y, a); \
        return hipGetLastError();                                                                            \
    }
        PO2Q_RKF(3, false) PO2Q_RKF(2, false) PO2Q_RKF(3, true) PO2Q_RKF(2, true)
#undef PO2Q_RKF
        return hipErrorInvalidValue;
    }
#define PO2Q_RK1(c, d, e, v, tt, lw)                                                                      \
    if (p.C == c && p.pd == d && epi == e && p.vrx == v && !p.nts) {                                         \
        hipLaunchKernelGGL((conv_rowsk<c, d, tt, lw, e>), dim3((unsigned)p.blocks), dim3(kThreads + (lw ? 64 : 0)), \
                           p.lds_bytes, s, x, reinterpret_cast<const uint4*>(packed), scale, bias, y, a);     \
        return hipGetLastError();                                                                            \
    }
#define PO2Q_RKN1(c, d, e, v, tt, lw, nt)                                                                 \
    if (p.C == c && p.pd == d && epi == e && p.vrx == v && p.nts == nt) {                                    \
        hipLaunchKernelGGL((conv_rowsk<c, d, tt, lw, e, 0, nt>), dim3((unsigned)p.blocks),                  \
                           dim3(kThreads + (lw ? 64 : 0)), p.lds_bytes, s, x, reinterpret_cast<const uint4*>(packed), \
                           scale, bias, y, a);                                                               \
        return hipGetLastError();                                                                            \
    }
#define PO2Q_RKN(c, d, e, v, tt, lw) \
    PO2Q_RKN1(c, d, e, v, tt, lw, 1) PO2Q_RKN1(c, d, e, v, tt, lw, 2) PO2Q_RKN1(c, d, e, v, tt, lw, 3)
#define PO2Q_RK(c, d, e) PO2Q_RK1(c, d, e, 1, false, false) PO2Q_RK1(c, d, e, 2, true, false)
    // the pipelined split (PIPE) for C = 64's MFMA-wave plans: default for the direct-store plans
    // (0.159 vs 0.182 ms at bs 256 @56), not for the TT plans (no change there:
    // profiles/r04_rowsk_pipe_ab.jsonl).  PO2Q_ROWSK_PIPE=0: never, 1: also with TT.
    const int pipe = [] {
        const char* e = getenv("PO2Q_ROWSK_PIPE");
        return e ? atoi(e) : -1;
    }();
#define PO2Q_RKP(d, e, v, tt)                                                                                \
    if ((pipe == 1 || (pipe < 0 && v == 1)) && p.C == 64 && p.pd == d && epi == e && p.vrx == v && !p.nts) { \
        hipLaunchKernelGGL((conv_rowsk<64, d, tt, false, e, 0, 0, false, false, true>), dim3((unsigned)p.blocks), \
                           dim3(kThreads), p.lds_bytes, s, x, reinterpret_cast<const uint4*>(packed), scale, bias, y, a); \
        return hipGetLastError();                                                                            \
    }
    PO2Q_RKP(2, false, 2, true) PO2Q_RKP(3, false, 2, true) PO2Q_RKP(2, true, 2, true) PO2Q_RKP(3, true, 2, true)
    PO2Q_RKP(2, false, 1, false) PO2Q_RKP(3, false, 1, false) PO2Q_RKP(2, true, 1, false) PO2Q_RKP(3, true, 1, false)
#undef PO2Q_RKP
    // ... and the direct-store plans with non-temporal stores / loads
#define PO2Q_RKPN1(d, e, nt)                                                                                 \
    if (pipe != 0 && p.C == 64 && p.pd == d && epi == e && p.vrx == 1 && p.nts == nt) {                      \
        hipLaunchKernelGGL((conv_rowsk<64, d, false, false, e, 0, nt, false, false, true>), dim3((unsigned)p.blocks), \
                           dim3(kThreads), p.lds_bytes, s, x, reinterpret_cast<const uint4*>(packed), scale, bias, y, a); \
        return hipGetLastError();                                                                            \
    }
#define PO2Q_RKPN(d, e) PO2Q_RKPN1(d, e, 1) PO2Q_RKPN1(d, e, 2) PO2Q_RKPN1(d, e, 3)
    PO2Q_RKPN(2, false) PO2Q_RKPN(3, false) PO2Q_RKPN(2, true) PO2Q_RKPN(3, true)
#undef PO2Q_RKPN
#undef PO2Q_RKPN1
#ifdef PO2Q_ROWS_DIAG
    if (const char* dv = getenv("PO2Q_ROWSK_DEBUG")) {
        const int dbg = atoi(dv);
#define PO2Q_RKD(c, d, tt, lw, v)                                                                          \
    if (dbg == v && p.C == c && p.pd == d && (p.vrx >= 2) == tt && (p.vrx == 3) == lw) {                   \
        hipLaunchKernelGGL((conv_rowsk<c, d, tt, lw, false, v>), dim3((unsigned)p.blocks), dim3(kThreads + (lw ? 64 : 0)), \
                           p.lds_bytes, s, x, reinterpret_cast<const uint4*>(packed), scale, bias, y, a);    \
        return hipGetLastError();                                                                           \
    }
#define PO2Q_RKDS(v) PO2Q_RKD(32, 3, true, false, v) PO2Q_RKD(32, 3, true, true, v)
        PO2Q_RKDS(6) PO2Q_RKDS(16) PO2Q_RKDS(2) PO2Q_RKDS(1) PO2Q_RKDS(7)
#undef PO2Q_RKDS
        // stage 3's TT plan (C = 64, 2 rows in flight)
#define PO2Q_RKDS(v) PO2Q_RKD(64, 2, true, false, v)
        PO2Q_RKDS(2) PO2Q_RKDS(4) PO2Q_RKDS(6) PO2Q_RKDS(16) PO2Q_RKDS(64) PO2Q_RKDS(128) PO2Q_RKDS(256)
        PO2Q_RKDS(144) PO2Q_RKDS(400) PO2Q_RKDS(404) PO2Q_RKDS(148) PO2Q_RKDS(20) PO2Q_RKDS(132)
#undef PO2Q_RKDS
#undef PO2Q_RKD
    }
#endif
    PO2Q_RK(64, 3, false) PO2Q_RK(64, 2, false) PO2Q_RK(32, 3, false) PO2Q_RK(32, 2, false)
    PO2Q_RK(64, 3, true) PO2Q_RK(64, 2, true) PO2Q_RK(32, 3, true) PO2Q_RK(32, 2, true)
    PO2Q_RK1(32, 3, false, 3, true, true) PO2Q_RK1(32, 3, true, 3, true, true)
    PO2Q_RKN(64, 3, false, 1, false, false) PO2Q_RKN(64, 2, false, 1, false, false)
    PO2Q_RKN(64, 3, true, 1, false, false) PO2Q_RKN(64, 2, true, 1, false, false)
    PO2Q_RKN(32, 3, false, 3, true, true) PO2Q_RKN(32, 3, true, 3, true, true)

#undef PO2Q_RK
#undef PO2Q_RK1
#undef PO2Q_RKN
#undef PO2Q_RKN1
    return hipErrorInvalidValue;
}

// The residual add inside the kernel (po2q_epi.h): the loader-wave plans of C = K = 32, and
// every C = K = 64 plan -- run as its TT sibling with 2 ring slots (the residual ring makes
// it 2 blocks per CU: 77 KiB of LDS) -- instead of the conv plus an elementwise pass over y
// (the BasicBlock conv2 of ResNet56 stage 3, reference models/resnet.py:69-71).
static bool rowsk64_res_on() {
    static const bool on = [] {
        const char* e = getenv("PO2Q_ROWSK_RES");
        return !(e && e[0] == '0');
    }();
    return on;
}

bool rowsk_res_ok(const ConvPlan& p) {
    if (p.kind != KIND_BF16X3_ROWS) return false;
    if (p.C == 32 && p.K == 32) return p.vrx == 3 && p.pd == 3 && !p.fp;
    return p.C == 64 && p.K == 64 && (p.vrx == 1 || p.vrx == 2) && rowsk64_res_on();
}

hipError_t launch_conv_rowsk_res(const ConvPlan& p, const float* x, const uint16_t* packed, const float* scale,
                                 const float* bias, float* y, const float* ps, const float* pb, const float* res,
                                 int act, hipStream_t s, const WQuant& q) {
    if (!rowsk_res_ok(p) || !res) return hipErrorInvalidValue;
    RowsKArgs a;
    a.N = p.N; a.H = p.H; a.W = p.W; a.P = p.P; a.Q = p.Q;
    a.RB = p.TP; a.nseg = p.tilesP; a.nstrip = p.tilesQ;
    a.items = p.N * p.tilesP * p.tilesQ;
    a.remap = (p.blocks % 8 == 0) ? 1 : 0;
    a.ps = ps;
    a.pb = pb;
    a.act = act;
    a.res = res;
    a.q = q;
    if (p.C == 64) {
        constexpr size_t lds64 = kKLds<64, 2, true> + 2 * kKTile<64>;
        if (p.fp) {
            if (!q.w) return hipErrorInvalidValue;
            hipLaunchKernelGGL((conv_rowsk<64, 2, true, false, true, 0, 0, true, true>), dim3((unsigned)p.blocks),
                               dim3(kThreads), lds64, s, x, reinterpret_cast<const uint4*>(packed), scale, bias, y, a);
        } else {
            hipLaunchKernelGGL((conv_rowsk<64, 2, true, false, true, 0, 0, true>), dim3((unsigned)p.blocks),
                               dim3(kThreads), lds64, s, x, reinterpret_cast<const uint4*>(packed), scale, bias, y, a);
        }
        return hipGetLastError();
    }
    const size_t lds = p.lds_bytes + 2 * kKTile<32>;
#define PO2Q_RKR(nt)                                                                                         \
    if (p.nts == nt) {                                                                                       \
        hipLaunchKernelGGL((conv_rowsk<32, 3, true, true, true, 0, nt, true>), dim3((unsigned)p.blocks),      \
                           dim3(kThreads + 64), lds, s, x, reinterpret_cast<const uint4*>(packed), scale, bias, y, a); \
        return hipGetLastError();                                                                            \
    }
    PO2Q_RKR(1) PO2Q_RKR(2) PO2Q_RKR(3)
#undef PO2Q_RKR
    if (p.nts != 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL((conv_rowsk<32, 3, true, true, true, 0, 0, true>), dim3((unsigned)p.blocks),
                       dim3(kThreads + 64), lds, s, x, reinterpret_cast<const uint4*>(packed), scale, bias, y, a);
    return hipGetLastError();
}

}  // namespace po2q
