// A chain of quantized 3x3 / stride-1 / pad-1 C -> C convs on SMALL images, all of them in ONE
// launch: the stride-1 run of a ResNet56 stage at CIFAR size (reference models/resnet.py:55-71,
// 25-50; each conv QuantizedConv2d.forward, models/quantized_conv.py:32-38), with each layer's
// eval BN affine, activation and the BasicBlock's identity shortcut in its store.
//
// Why: at 32x32 / 16x16 / 8x8 a layer is 4-17 MB and its arithmetic a microsecond or two of
// MFMA time per CU, so one launch per layer spends most of its ~10 us in the launch, the first
// load's latency, the store drain -- and, even in one launch, in the global round trip of every
// activation (profiles/r03_cifar32_chain_kernel_stats.csv: the single-layer autotune
// candidates).  Images are independent through the whole stage, so a block owns ONE image for
// every layer, and the activation never leaves the CU:
//   start:      x -> exact hi / mid / lo bf16 split planes [(H + 2) x (W + 2) padded pixels][C]
//               in LDS (zero halo), one batch of independent loads per thread;
//   per layer:  every wave computes ALL its 16-pixel groups' accumulators for its 16-channel
//               output tile (B fragments from the layer's pack, the row-kernel layout; the
//               transposed MFMA form, so a lane ends with 4 consecutive channels of one pixel),
//               barrier (every read of the input planes retired), epilogue (bias, eval BN
//               affine, + the held residual, activation), split, and the planes are overwritten
//               IN PLACE (3 ds_write_b64), barrier; the last layer stores y instead.
//   residual:   a BasicBlock's input is held in VGPRs by the lanes that add it two layers later
//               (every layer maps (wave, lane) to the same pixel and channels).
// The weights of all layers are quantized + packed by batched pack launches first.  Same
// arithmetic as every bf16x3 kernel (exact +-2^e bf16 weights, exact 3-way split of the fp32
// activations -- each layer's fp32 output re-split exactly --, fp32 accumulation on
// v_mfma_f32_16x16x32_bf16).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "../../include/po2q.h"
#ifdef PO2Q_CHAIN_STAMPS
#include <cstdio>
#endif
#include "po2q_epi.h"
#include "po2q_internal.h"
#include "po2q_x3_dev.h"

namespace po2q {

namespace {
constexpr int kChainThreads = 512;  // 8 waves: two per SIMD
constexpr int kChainItems = 5;      // split items (pixel x channel octet) per thread and load batch
constexpr int kChainMax = PO2Q_CHAIN_MAX_LAYERS;
constexpr size_t kChainLdsMax = 160 * 1024;

// Byte offset of channel octet oc of padded pixel pp (padded column col) in a plane: the
// conflict-free swizzle of po2q_conv_img.hip (every ds_read_b128 lane group of a fragment read
// hits 64 distinct banks when a 16-pixel group is 16 consecutive pixels).  W8 (C = 64, W = 8: a
// group is two 8-pixel row pieces 10 padded pixels apart): the octet XORed with a per-column
// table instead (exhaustive search over every tap offset, tools-free: 3 bits per column).
template <int C, bool W8 = false>
__device__ __forceinline__ int ch_addr(int pp, int col, int oc) {
    if constexpr (C == 16) {
        // [pixel][octet]: pixels p and p + 8 of a group share banks (PMC: 34 % of the LDS cycles
        // conflicted, profiles/r05_pmc_chain16.json), yet both swizzles tried (octet flipped with pixel
        // bit 3; octet-major planes) were slower in the kernel: config 2 813k -> 759k img/s
        // (r05_ab_chain_bit3.jsonl, r05_ab_chain_octet_major.jsonl)
        return pp * 32 + 16 * oc;
    } else if constexpr (C == 32) {
        return pp * 64 + 16 * (oc ^ (((pp >> 2) & 1) << 1));
    } else if constexpr (W8) {
        return pp * 128 + 16 * (oc ^ (int)((0x53e0e1u >> (3 * (col & 7))) & 7u));
    } else {
        return pp * 128 + 16 * (oc ^ (((pp >> 1) & 3) << 1));
    }
}

size_t chain_plane(int64_t C, int64_t H, int64_t W) { return (size_t)((H + 2) * (W + 2) * 2 * C + 16); }

// f(integral_constant<int, i>) for i = 0 .. N-1, unrolled at compile time
template <class F, int... I>
__device__ __forceinline__ void static_for_impl(F& f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F& f) {
    static_for_impl(f, std::make_integer_sequence<int, N>{});
}
}  // namespace

struct ChainLayer {
    const uint4* wp;      // packed B fragments [r][ks][nt][lane] (row-kernel layout)
    const float* scale;   // the layer's max|w| multiplier
    const float* bias;    // [C] or NULL
    const float* ps;      // eval BN affine [C] or NULL
    const float* pb;
    int act;              // PO2Q_ACT_*
    int res_add;          // 1: + the held residual (a BasicBlock's input) before the activation
    int keep;             // 1: this layer's output is a later layer's residual: hold it
};

struct ChainArgs {
    int H, W, L;
    int PW, PL, ZO;
    int res0;             // 1: x itself is a later layer's residual: hold it
    unsigned* stamps;     // PO2Q_CHAIN_STAMPS diagnostic builds only: per (block, wave) phase cycle sums
    ChainLayer layer[kChainMax];
};

// Diagnostic build (-DPO2Q_CHAIN_STAMPS, `make chainstamps`): s_memtime phase stamps, never in the
// product build.  Phases per layer: 0 loop top, 1 MFMA, 2 barrier after the MFMAs, 3 epilogue,
// 4 barrier after the epilogue; once: 5 x loads + split, 6 residual loads, 7 the prologue's barrier.
#ifdef PO2Q_CHAIN_STAMPS
#define CHS(i)                                                                           \
    do {                                                                                 \
        __builtin_amdgcn_sched_barrier(0);                                               \
        unsigned long long t_;                                                           \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");        \
        __builtin_amdgcn_sched_barrier(0);                                               \
        ph_[i] += (unsigned)(t_ - tprev_);                                               \
        tprev_ = t_;                                                                     \
    } while (0)
#else
#define CHS(i) \
    do {       \
    } while (0)
#endif


// Packed fp32 (v_pk_fma / v_pk_add) in the epilogue and its exact split: on by default here (same
// IEEE results either way; 1-2 % faster in the chain, 3 of 3 same-box rounds,
// profiles/r04_chain_pk_ab.jsonl -- unlike the conv pair, po2q_conv_pair.hip); -DPO2Q_CHAIN_PK=0
// builds the scalar form
#ifndef PO2Q_CHAIN_PK
#define PO2Q_CHAIN_PK 1
#endif
constexpr bool kChainPK = PO2Q_CHAIN_PK != 0;

// C: channels; MG: most 16-pixel groups one wave owns (register arrays).  The activation lives
// in LDS as split planes for the whole chain: per layer every wave first computes ALL its
// groups' accumulators (transposed MFMA form, A = weights, B = pixels: each lane ends with 4
// consecutive output channels of one pixel), a barrier retires every read of the layer's input,
// then the epilogue overwrites the planes in place (ds_write_b64 of 4 bf16 per plane) -- or, in
// the last layer, stores y.  A residual source (a BasicBlock's input) is held in VGPRs by the
// lanes that will add it: every layer maps (wave, lane) to the same (pixel, channels).
// FULL: every wave owns exactly MG whole groups (H * W a multiple of 16 * waves per tile * MG):
// no per-group bounds checks (the CIFAR stages).
// DB (C = 32 / 64): two plane sets, layer l reads set l & 1 and writes set (l + 1) & 1, so the
// barrier between a layer's MFMA phase and its epilogue goes: a wave's epilogue runs under the
// other waves' MFMAs, one barrier per layer.
template <int C, int MG, bool W8 = false, bool FULL = false, bool DB = false>
__global__ __launch_bounds__(kChainThreads, 1) void conv_chain(const float* __restrict__ x, float* __restrict__ y,
                                                               ChainArgs a) {
    constexpr int KS = C == 16 ? 2 : 3 * (C / 32);  // k-steps per tap row
    constexpr int NO = C / 8;                       // channel octets per pixel
    constexpr int NT = C / 16;                      // output tiles
    constexpr int WPT = (kChainThreads / 64) / NT;  // waves per output tile
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
#ifdef PO2Q_CHAIN_STAMPS
    unsigned ph_[8] = {};
    unsigned long long tprev_;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(tprev_)::"memory");
#endif
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int n = blockIdx.x;
    const int nt = wave % NT, gsub = wave / NT;
    const int H = a.H, W = a.W, PW = a.PW, HW = H * W;
    const int ngroups = (HW + 15) >> 4;
    const int p = lane & 15, g4 = lane >> 4;
    const int c0 = 16 * nt + 4 * g4;  // this lane's 4 output channels (transposed form)
    const int64_t img = (int64_t)C * HW;
    const float* xn = x + (int64_t)n * img;
    float* yn = y + (int64_t)n * img;

    // ---- x -> split planes, the zero halo with it (written once: later layers write interiors)
    const int nitems = (H + 2) * PW * NO;
    for (int base = 0; base < nitems; base += kChainThreads * kChainItems) {
        uint32_t v[kChainItems][8];
        int dst[kChainItems];
#pragma unroll
        for (int i = 0; i < kChainItems; ++i) {
            const int it = base + i * kChainThreads + tid;
            const bool ok = it < nitems;
            const int pc = it % PW, t = it / PW;
            const int rr = t % (H + 2), oc = t / (H + 2);
            const int h = rr - 1, xc = pc - 1;
            const bool inb = ok && h >= 0 && h < H && xc >= 0 && xc < W;
            const float* src = xn + (int64_t)(8 * oc) * HW + (inb ? h * W + xc : 0);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[i][e] = inb ? __float_as_uint(src[(int64_t)e * HW]) : 0u;
            dst[i] = ok ? ch_addr<C, W8>(rr * PW + pc, pc, oc) : -1;
        }
#pragma unroll
        for (int i = 0; i < kChainItems; ++i) {
            if (dst[i] < 0) continue;
            uint4 hi, mid, lo;
            split3(v[i], hi, mid, lo);
            *reinterpret_cast<uint4*>(lds + dst[i]) = hi;
            *reinterpret_cast<uint4*>(lds + a.PL + dst[i]) = mid;
            *reinterpret_cast<uint4*>(lds + 2 * a.PL + dst[i]) = lo;
        }
    }
    CHS(5);
    if (tid < 3) *reinterpret_cast<uint4*>(lds + tid * a.PL + a.ZO) = make_uint4(0u, 0u, 0u, 0u);
    if constexpr (DB) {  // the second set's zero halo (and zero slot): the whole set zeroed once
        for (int i = tid; i < 3 * a.PL / 16; i += kChainThreads)
            *reinterpret_cast<uint4*>(lds + 3 * a.PL + 16 * i) = make_uint4(0u, 0u, 0u, 0u);
    }
    // the held residual: x itself when a later layer adds it
    float rres[MG][4];
#pragma unroll
    for (int gi = 0; gi < MG; ++gi) {
        const int f = 16 * (gsub + gi * WPT) + p;
        const bool ok = a.res0 && f < HW;
#pragma unroll
        for (int i = 0; i < 4; ++i) rres[gi][i] = ok ? xn[(int64_t)(c0 + i) * HW + f] : 0.0f;
    }
    // ---- the layer descriptors (kernel arguments read with scalar loads at the top of every layer):
    // one batch of scalar loads over every 64-byte line of the arguments and ONE wait, here where the
    // residual loads are in flight, so the per-layer descriptor reads hit the scalar cache instead of
    // each paying a cold miss
    {
        static_assert(offsetof(ChainArgs, layer) + sizeof(ChainLayer) * kChainMax + 16 <= 22 * 64,
                      "the warm-up below covers 22 whole 64-byte lines of kernel arguments");
        const auto kp = __builtin_amdgcn_kernarg_segment_ptr();
        unsigned d;
#define PO2Q_WL(o) "s_load_dword %0, %1, " #o "\n\t"
        asm volatile(PO2Q_WL(0x0) PO2Q_WL(0x40) PO2Q_WL(0x80) PO2Q_WL(0xc0) PO2Q_WL(0x100) PO2Q_WL(0x140)
                     PO2Q_WL(0x180) PO2Q_WL(0x1c0) PO2Q_WL(0x200) PO2Q_WL(0x240) PO2Q_WL(0x280) PO2Q_WL(0x2c0)
                     PO2Q_WL(0x300) PO2Q_WL(0x340) PO2Q_WL(0x380) PO2Q_WL(0x3c0) PO2Q_WL(0x400) PO2Q_WL(0x440)
                     PO2Q_WL(0x480) PO2Q_WL(0x4c0) PO2Q_WL(0x500) PO2Q_WL(0x540) "s_waitcnt lgkmcnt(0)"
                     : "=&s"(d)
                     : "s"(kp)
                     : "memory");
#undef PO2Q_WL
        (void)d;
    }
    CHS(6);
    __syncthreads();
    CHS(7);

    // this wave's groups: padded pixel of tap (0, 0) per group (past the image: pixel 0, the
    // result is not stored -- every group runs the same unrolled MFMA sequence)
    int pp0[MG], px0[MG];
#pragma unroll
    for (int gi = 0; gi < MG; ++gi) {
        const int grp = gsub + gi * WPT;
        const int f = 16 * grp + p;
        const int fo = (FULL || (grp < ngroups && f < HW)) ? f : 0;
        const int oy = fo / W;
        px0[gi] = fo - oy * W;
        pp0[gi] = oy * PW + px0[gi];
    }
    // A-fragment (pixel) address of step st = (group, tap row r, k-step ks) in a plane
    auto a_addr = [&](auto ST_) __attribute__((always_inline)) {
        constexpr int st = decltype(ST_)::value;
        constexpr int gi = st / (3 * KS), t = st % (3 * KS), r = t / KS, ks = t % KS;
        if constexpr (C == 16) {
            const int s = ks == 0 ? (g4 >> 1) : 2;
            return (ks == 1 && g4 >= 2) ? a.ZO : ch_addr<C, W8>(pp0[gi] + r * PW + s, px0[gi] + s, g4 & 1);
        } else {
            return ch_addr<C, W8>(pp0[gi] + r * PW + ks % 3, px0[gi] + ks % 3, (ks / 3) * 4 + g4);
        }
    };
    constexpr int T = 3 * KS;    // MFMA steps (x 3 planes) per group
    constexpr int S = MG * T;    // steps per layer
    constexpr int PD = 4;        // A-fragment reads issued this many steps ahead (3 each: lgkmcnt <= 12)

    // the first layer's B fragments (later layers': prefetched behind the previous layer's MFMAs,
    // straight into the registers the next MFMAs read -- no loop-carried copy to wait for)
    bf16x8 bw[3 * KS];
    auto load_bw = [&](const ChainLayer& ly) __attribute__((always_inline)) {
#pragma unroll
        for (int f = 0; f < 3 * KS; ++f) bw[f] = __builtin_bit_cast(bf16x8, ly.wp[(f * NT + nt) * 64 + lane]);
    };
    load_bw(a.layer[0]);

    // C = 16: the 27 sixteen-channel units of an output pixel (3 tap rows x 3 taps x 3 planes) in 14
    // k-steps instead of 18: per tap row (s0 | s1) of each plane (9 steps), then the nine s2 units
    // paired across planes AND tap rows -- every tap row feeds the same accumulator here --:
    // (r0 hi | r0 mid), (r0 lo | r1 hi), (r1 mid | r1 lo), (r2 hi | r2 mid), (r2 lo | zero).  The
    // pairs' B fragments hold the s2 weights of the two tap rows in their two k-halves; they are
    // built per layer from the pack's (s2 | zero) fragments with v_permlane32_swap (lanes 32-63 of
    // a fragment take lanes 0-31 of the other).  One plane read per MFMA, issued PD16 steps ahead;
    // FULL (the CIFAR stages) orders the MFMAs k-step major, so consecutive MFMAs accumulate into
    // different groups (the group-major order of the other shapes keeps them under 256 VGPRs).
    auto mma16 = [&](floatx4 (&acc)[MG]) __attribute__((always_inline)) {
        constexpr int T1 = 14, S1 = MG * T1, PD16 = 10;
        bf16x8 bq[8];
        auto pair = [&](const bf16x8& lo, const bf16x8& hi) __attribute__((always_inline)) {
            const uint4 u = __builtin_bit_cast(uint4, lo), v = __builtin_bit_cast(uint4, hi);
            uint4 r;
            r.x = __builtin_amdgcn_permlane32_swap(u.x, v.x, false, false)[0];
            r.y = __builtin_amdgcn_permlane32_swap(u.y, v.y, false, false)[0];
            r.z = __builtin_amdgcn_permlane32_swap(u.z, v.z, false, false)[0];
            r.w = __builtin_amdgcn_permlane32_swap(u.w, v.w, false, false)[0];
            return __builtin_bit_cast(bf16x8, r);
        };
        bq[0] = bw[0];
        bq[1] = bw[2];
        bq[2] = bw[4];
        bq[3] = pair(bw[1], bw[1]);  // (r0 hi | r0 mid)
        bq[4] = pair(bw[1], bw[3]);  // (r0 lo | r1 hi)
        bq[5] = pair(bw[3], bw[3]);  // (r1 mid | r1 lo)
        bq[6] = pair(bw[5], bw[5]);  // (r2 hi | r2 mid)
        bq[7] = bw[5];               // (r2 lo | zero)
        // Addresses: the unswizzled C = 16 plane is linear in the pixel (32 bytes each), so a read is
        // one VGPR add: a per-group lane base plus a uniform offset (tap row, plane; SGPR) for the
        // (s0 | s1) steps, or plus a per-lane offset (the two k-halves' tap rows / planes) for the
        // paired s2 steps.  The last pair's zero half reads the r2 lo unit again (finite: the split
        // clamps mid / lo) against zero weights, so it needs no zero slot.
        constexpr int PXB = 32;
        const int OCB = 16;
        int lb[MG], dsel[5];
#pragma unroll
        for (int gi = 0; gi < MG; ++gi) lb[gi] = (pp0[gi] + 2) * PXB + OCB * (g4 & 1);  // tap s = 2
#pragma unroll
        for (int u = 0; u < 5; ++u) {
            const int ua = 2 * u, ub = u == 4 ? 8 : 2 * u + 1;
            const int ra = ua / 3, pa = ua % 3, rb = ub / 3, pb = ub % 3;
            dsel[u] = g4 < 2 ? ra * PW * PXB + pa * a.PL : rb * PW * PXB + pb * a.PL;
        }
        const int s01 = ((g4 >> 1) - 2) * PXB;  // tap (g4 >> 1) relative to the s = 2 base
        auto addr = [&](auto ST_) __attribute__((always_inline)) {
            constexpr int st = decltype(ST_)::value;
            constexpr int t = FULL ? st / MG : st % T1, gi = FULL ? st % MG : st / T1;  // FULL: k-step major
            if constexpr (t < 9) {
                constexpr int r = t / 3, pl = t % 3;
                return lb[gi] + s01 + (r * PW * PXB + pl * a.PL);
            } else {
                return lb[gi] + dsel[t - 9];
            }
        };
        bf16x8 ring[PD16 + 1];
        auto issue = [&](auto ST_) __attribute__((always_inline)) {
            constexpr int st = decltype(ST_)::value;
            if constexpr (st < S1)
                ring[st % (PD16 + 1)] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(lds + addr(ST_)));
        };
        auto step = [&](auto ST_) __attribute__((always_inline)) {
            constexpr int st = decltype(ST_)::value;
            issue(std::integral_constant<int, st + PD16>{});
            constexpr int t = FULL ? st / MG : st % T1, gi = FULL ? st % MG : st / T1;  // FULL: k-step major
            constexpr int bi = t < 9 ? t / 3 : 3 + (t - 9);
            acc[gi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[bi], ring[st % (PD16 + 1)], acc[gi], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        };
        static_for<PD16>(issue);
        static_for<S1>(step);
    };

    for (int l = 0; l < a.L; ++l) {
        const ChainLayer ly = a.layer[l];  // one batch of scalar loads for the whole descriptor
        const int rd = DB ? (l & 1) * 3 * a.PL : 0, wr = DB ? ((l + 1) & 1) * 3 * a.PL : 0;
        // this layer's epilogue constants: loaded now, consumed after the MFMA phase
        const float scale = *ly.scale;
        // one uniform branch per vector (a per-element test had put 12 scalar branches in the loop top)
        float cbk[4] = {0.f, 0.f, 0.f, 0.f}, ceps[4] = {1.f, 1.f, 1.f, 1.f}, cepb[4] = {0.f, 0.f, 0.f, 0.f};
        if (ly.bias) {
#pragma unroll
            for (int i = 0; i < 4; ++i) cbk[i] = ly.bias[c0 + i];
        }
        if (ly.ps) {
#pragma unroll
            for (int i = 0; i < 4; ++i) ceps[i] = ly.ps[c0 + i];
        }
        if (ly.pb) {
#pragma unroll
            for (int i = 0; i < 4; ++i) cepb[i] = ly.pb[c0 + i];
        }
        // opaque per layer: keeps the step addresses from being hoisted out of the layer loop
        // (one VGPR per step held across every layer)
#pragma unroll
        for (int gi = 0; gi < MG; ++gi) asm volatile("" : "+v"(pp0[gi]), "+v"(px0[gi]));
        // ---- every group's accumulator (the planes are read-only in this phase), software-
        // pipelined: the 3 plane reads of step st + PD go out before the MFMAs of step st
        floatx4 acc[MG];
#pragma unroll
        for (int gi = 0; gi < MG; ++gi) acc[gi] = floatx4{0.f, 0.f, 0.f, 0.f};
        CHS(0);
        if constexpr (C == 16) {
            mma16(acc);
        } else {
        bf16x8 ring[PD + 1][3];
        auto issue = [&](auto ST_) __attribute__((always_inline)) {
            constexpr int st = decltype(ST_)::value;
            if constexpr (st < S) {
                const int ad = a_addr(ST_);
#pragma unroll
                for (int pl = 0; pl < 3; ++pl)
                    ring[st % (PD + 1)][pl] =
                        __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(lds + rd + pl * a.PL + ad));
            }
        };
        auto step = [&](auto ST_) __attribute__((always_inline)) {
            constexpr int st = decltype(ST_)::value;
            issue(std::integral_constant<int, st + PD>{});
            constexpr int gi = st / T, t = st % T;
            const bf16x8 bb = bw[t];  // t = r * KS + ks: the pack's fragment order
#pragma unroll
            for (int pl = 0; pl < 3; ++pl)  // transposed: D[out channel][pixel]
                acc[gi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bb, ring[st % (PD + 1)][pl], acc[gi], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        };
        static_for<PD>(issue);
        static_for<S>(step);
        }

        // the next layer's B fragments go out now (the last layer reloads its own: no branch, so
        // the epilogue's wait for this layer's constants stays a counted vmcnt, not vmcnt(0))
        CHS(1);
        const bool last = l + 1 == a.L;
        const int act = ly.act, res_add = ly.res_add, keep = ly.keep;
        load_bw(a.layer[last ? l : l + 1]);
        // every read of this layer's input planes has retired.  A bare s_barrier, not
        // __syncthreads: its release fence would wait for the prefetches just issued (vmcnt(0)).
        // DB: the epilogue writes the other set, nothing to wait for
        if constexpr (!DB) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
        }
        CHS(2);

        // ---- epilogue: lane = channels c0 .. c0 + 3 of pixel 16 grp + p.  The activation and the
        // residual add are compile-time inside (one dispatch per layer): a runtime activation switch
        // per value had put ~6 scalar branches beside every value (the epilogue took 1.3x the MFMA
        // phase, profiles/r04_chain_stamps.txt)
        auto epilogue = [&](auto ACT_, auto RA_) __attribute__((always_inline)) {
            constexpr int ACT = decltype(ACT_)::value;
            constexpr bool RA = decltype(RA_)::value;
#pragma unroll
            for (int gi = 0; gi < MG; ++gi) {
                const int grp = gsub + gi * WPT;
                const int f = 16 * grp + p;
                if (!FULL && (grp >= ngroups || f >= HW)) continue;
                float v[4];
#pragma unroll
                for (int i = 0; i < 4; i += 2) {  // channel pairs as packed v_pk_fma / v_pk_add (the same IEEE ops)
                    if constexpr (!kChainPK) {
#pragma unroll
                        for (int e = i; e < i + 2; ++e) {
                            float u = (acc[gi][e] * scale + cbk[e]) * ceps[e] + cepb[e];
                            if constexpr (RA) u += rres[gi][e];
                            v[e] = epi_act_ct<ACT>(u);
                        }
                        continue;
                    }
                    const po2q_float2 sc = {scale, scale};
                    po2q_float2 u = (po2q_float2{acc[gi][i], acc[gi][i + 1]} * sc + po2q_float2{cbk[i], cbk[i + 1]}) *
                                        po2q_float2{ceps[i], ceps[i + 1]} +
                                    po2q_float2{cepb[i], cepb[i + 1]};
                    if constexpr (RA) u += po2q_float2{rres[gi][i], rres[gi][i + 1]};
                    v[i] = epi_act_ct<ACT>(u.x);
                    v[i + 1] = epi_act_ct<ACT>(u.y);
                }
                if (keep) {  // wave-uniform
#pragma unroll
                    for (int e = 0; e < 4; ++e) rres[gi][e] = v[e];
                }
                if (last) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) yn[(int64_t)(c0 + i) * HW + f] = v[i];
                } else {
                    // padded pixel (oy + 1, ox + 1) of output pixel f = (oy, ox): pp0 / px0 hold (oy, ox) of
                    // tap (0, 0), so no division by W here
                    const int ad = ch_addr<C, W8>(pp0[gi] + PW + 1, px0[gi] + 1, c0 >> 3) + 8 * ((c0 >> 2) & 1);
                    uint2 hi, mid, lo;
                    const uint32_t vb[4] = {__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]),
                                            __float_as_uint(v[3])};
                    split4p<kChainPK>(vb, hi, mid, lo);
                    *reinterpret_cast<uint2*>(lds + wr + ad) = hi;
                    *reinterpret_cast<uint2*>(lds + wr + a.PL + ad) = mid;
                    *reinterpret_cast<uint2*>(lds + wr + 2 * a.PL + ad) = lo;
                }
            }
        };
        with_act(act, [&](auto ACT_) __attribute__((always_inline)) {
            if (res_add)
                epilogue(ACT_, std::true_type{});
            else
                epilogue(ACT_, std::false_type{});
        });
        CHS(3);
        // the next layer's input planes are complete (the block's own LDS writes: lgkmcnt)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        CHS(4);
    }
#ifdef PO2Q_CHAIN_STAMPS
    if (lane == 0 && a.stamps)
        for (int i = 0; i < 8; ++i) a.stamps[((size_t)blockIdx.x * 8 + wave) * 8 + i] = ph_[i];
#endif
}

// ------------------------------------------------------------------- host side --
// most 16-pixel groups one wave owns: ceil(ceil(HW / 16) / waves per output tile); the register
// arrays take up to 8 (C = 16: 32x32) or 4 (C = 32: 16x16, C = 64: 8x16) without spilling
static int chain_mg(int64_t C, int64_t H, int64_t W) {
    const int64_t groups = (H * W + 15) / 16, wpt = (kChainThreads / 64) / (C / 16);
    return (int)((groups + wpt - 1) / wpt);
}
static int chain_mg_max(int64_t C) { return C == 16 ? 8 : 4; }

static bool chain_geom_ok(int64_t N, int64_t C, int64_t H, int64_t W, int n_layers) {
    if (!(C == 16 || C == 32 || C == 64) || N < 1 || H < 1 || W < 4 || W % 4 != 0) return false;
    if (n_layers < 1 || n_layers > kChainMax || N > INT32_MAX) return false;
    if (N * C * H * W >= (1LL << 40) || chain_mg(C, H, W) > chain_mg_max(C)) return false;
    return 3 * chain_plane(C, H, W) <= kChainLdsMax;
}

static bool chain_mode_ok(int bits, int fsr, int mode) {
    if (mode != PO2Q_MODE_PO2 && mode != PO2Q_MODE_PO2_PLUS) return false;
    if (bits < 1 || bits > 16) return false;
    const long lo = (long)fsr - (1L << (bits - 1)), hi = (long)fsr - 1;
    return lo >= -126 && hi <= 127;  // +-2^e must be a normal bf16
}

// The pack geometry of one layer (the small-image kernel's row layout).
static ConvPlan chain_plan(int64_t N, int64_t C, int64_t H, int64_t W) {
    ConvPlan p{};
    p.N = (int)N; p.C = (int)C; p.H = (int)H; p.W = (int)W; p.K = (int)C;
    p.R = p.S = 3; p.sh = p.sw = 1; p.ph = p.pw = 1; p.dh = p.dw = 1; p.groups = 1;
    p.P = p.H; p.Q = p.W; p.Cg = p.C; p.Kg = p.K;
    p.kind = KIND_BF16X3_IMG;
    p.CC = C == 16 ? 16 : 32;
    p.nchunks = (int)C / p.CC;
    p.steps = C == 16 ? 2 : 3 * p.nchunks;
    p.NT = (int)C / 16;
    p.taps = 9;
    p.packed_floats = (int64_t)3 * p.steps * p.NT * 64 * 4;
    return p;
}

namespace {
constexpr size_t kChainAlign = 256;
size_t chain_align(size_t v) { return (v + kChainAlign - 1) / kChainAlign * kChainAlign; }
struct ChainWs {
    size_t packed_off, packed_bytes, scale_off, total;
};
ChainWs chain_ws(int64_t N, int64_t C, int64_t H, int64_t W, int n_layers) {
    ChainWs L;
    const ConvPlan p = chain_plan(N, C, H, W);
    L.packed_bytes = chain_align((size_t)p.packed_floats * 4);
    L.packed_off = 0;
    L.scale_off = L.packed_bytes * (size_t)n_layers;
    L.total = L.scale_off + chain_align((size_t)n_layers * 4);
    return L;
}
}  // namespace

}  // namespace po2q

using namespace po2q;

extern "C" {

int po2q_qconv2d_chain_supported(int64_t N, int64_t C, int64_t H, int64_t W, int n_layers, int bits, int fsr,
                                 int mode) {
    return chain_geom_ok(N, C, H, W, n_layers) && chain_mode_ok(bits, fsr, mode) ? 1 : 0;
}

size_t po2q_qconv2d_chain_workspace_bytes(int64_t N, int64_t C, int64_t H, int64_t W, int n_layers) {
    if (!chain_geom_ok(N, C, H, W, n_layers)) return 0;
    return chain_ws(N, C, H, W, n_layers).total;
}

int po2q_qconv2d_chain_f32(const float* x, const float* const* w, const float* const* bias,
                           const float* const* post_scale, const float* const* post_shift, const int* act,
                           const int* res_from, int n_layers, int64_t N, int64_t C, int64_t H, int64_t W, int bits,
                           int fsr, int mode, float* y, void* workspace, size_t workspace_bytes, void* stream) {
    if (!chain_geom_ok(N, C, H, W, n_layers)) {
        set_error("po2q: chain needs C in {16, 32, 64}, W % 4 == 0, 1.." + std::to_string(kChainMax) +
                  " layers and a small image: its split planes in LDS ((H + 2)(W + 2) 6C bytes <= 160 KiB) and "
                  "at most 8 (C = 16) / 4 (C = 32, 64) 16-pixel groups per wave");
        return PO2Q_ERR_INVALID;
    }
    if (!chain_mode_ok(bits, fsr, mode)) {
        set_error("po2q: chain needs mode po2 / po2+ with exponents in the bf16 range");
        return PO2Q_ERR_INVALID;
    }
    if (!x || !w || !y || !workspace) {
        set_error("po2q: chain: null pointer");
        return PO2Q_ERR_INVALID;
    }
    const ChainWs L = chain_ws(N, C, H, W, n_layers);
    if (workspace_bytes < L.total) {
        set_error("po2q: chain workspace too small (need " + std::to_string(L.total) + " bytes)");
        return PO2Q_ERR_WORKSPACE;
    }
    for (int l = 0; l < n_layers; ++l) {
        if (!w[l]) {
            set_error("po2q: chain: null weight of layer " + std::to_string(l));
            return PO2Q_ERR_INVALID;
        }
        const int ac = act ? act[l] : 0;
        if (ac < 0 || ac > 3) {
            set_error("po2q: chain: unknown activation of layer " + std::to_string(l));
            return PO2Q_ERR_INVALID;
        }
        const int r = res_from ? res_from[l] : -1;
        if (r < -1 || r > l) {
            set_error("po2q: chain: res_from[" + std::to_string(l) + "] must be -1 or a layer index <= " +
                      std::to_string(l) + " (the residual is that layer's input)");
            return PO2Q_ERR_INVALID;
        }
    }
    // residual sources are held in VGPRs, one at a time: the intervals [source, user] of two
    // different sources must not overlap (a BasicBlock chain: [2b, 2b + 1] per block)
    for (int l1 = 0; l1 < n_layers; ++l1)
        for (int l2 = l1 + 1; l2 < n_layers; ++l2) {
            const int r1 = res_from ? res_from[l1] : -1, r2 = res_from ? res_from[l2] : -1;
            if (r1 >= 0 && r2 >= 0 && r1 != r2 && r2 <= l1) {
                set_error("po2q: chain: res_from holds one residual source at a time (layers " + std::to_string(l1) +
                          " and " + std::to_string(l2) + " add different, overlapping sources)");
                return PO2Q_ERR_INVALID;
            }
        }
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    char* ws = reinterpret_cast<char*>(workspace);

    // every layer's weight: quantize + pack in ceil(n / 36) launches
    const ConvPlan plan = chain_plan(N, C, H, W);
    std::vector<const ConvPlan*> plans((size_t)n_layers, &plan);
    std::vector<uint16_t*> packed((size_t)n_layers);
    std::vector<float*> scales((size_t)n_layers);
    for (int l = 0; l < n_layers; ++l) {
        packed[l] = reinterpret_cast<uint16_t*>(ws + L.packed_off + (size_t)l * L.packed_bytes);
        scales[l] = reinterpret_cast<float*>(ws + L.scale_off) + l;
    }
    hipError_t he = launch_pack_bf16x3_batch(n_layers, plans.data(), w, packed.data(), scales.data(), bits, fsr,
                                             mode, s);
    if (he != hipSuccess) {
        set_error(std::string("po2q: chain weight pack launch: ") + hipGetErrorString(he));
        return PO2Q_ERR_HIP;
    }

    std::vector<int> used((size_t)n_layers + 1, 0);  // input of layer j is a residual source
    for (int l = 0; l < n_layers; ++l)
        if (res_from && res_from[l] >= 0) used[res_from[l]] = 1;
    ChainArgs a{};
    a.stamps = nullptr;
    a.H = (int)H; a.W = (int)W; a.L = n_layers;
    a.PW = (int)W + 2;
    a.PL = (int)chain_plane(C, H, W);
    a.ZO = a.PL - 16;
    a.res0 = used[0];
    for (int l = 0; l < n_layers; ++l) {
        ChainLayer& ly = a.layer[l];
        ly.wp = reinterpret_cast<const uint4*>(packed[l]);
        ly.scale = scales[l];
        ly.bias = bias ? bias[l] : nullptr;
        ly.ps = post_scale ? post_scale[l] : nullptr;
        ly.pb = post_shift ? post_shift[l] : nullptr;
        ly.act = act ? act[l] : 0;
        ly.res_add = (res_from && res_from[l] >= 0) ? 1 : 0;
        ly.keep = used[l + 1];
    }
    // PO2Q_CHAIN_VARIANT (test knob): bit 0 the checked form everywhere, bit 3 one plane set.  Default: double-buffered planes for C = 32 / 64 (two sets
    // fit): 0.0849 vs 0.0861 ms at 32 x 16^2 and 0.0782 vs 0.0795 at 64 x 8^2, 17 layers bs 256,
    // 5 of 5 interleaved rounds (profiles/r04_chain_ab_db.jsonl)
    const char* venv = getenv("PO2Q_CHAIN_VARIANT");
    const int variant = venv ? atoi(venv) : 0;
    const bool db = !(variant & 8) && C != 16 && 6 * (size_t)a.PL <= kChainLdsMax;
    const size_t lds = (db ? 6 : 3) * (size_t)a.PL;
    const dim3 grid((unsigned)N), block(kChainThreads);
    const int mg = chain_mg(C, H, W);
    const bool w8 = C == 64 && W == 8;
    const int64_t wpt = (kChainThreads / 64) / (C / 16);
    const bool full = !(variant & 1) && (H * W) % 16 == 0 && (H * W / 16) % wpt == 0;
    // the exact-fit forms (FULL) for the CIFAR stages, the checked forms for everything else
    auto launch = [&](const ChainArgs& a) -> bool {
#define PO2Q_CH(c, m, w)                                                                               \
    if (C == c && mg <= m && w8 == w) {                                                                \
        if (c != 16 && db) {                                                                           \
            if (full && mg == m)                                                                       \
                hipLaunchKernelGGL((conv_chain<c, m, w, true, true>), grid, block, lds, s, x, y, a);   \
            else                                                                                       \
                hipLaunchKernelGGL((conv_chain<c, m, w, false, true>), grid, block, lds, s, x, y, a);  \
        } else if (full && mg == m) {                                                                  \
            hipLaunchKernelGGL((conv_chain<c, m, w, true>), grid, block, lds, s, x, y, a);            \
        } else {                                                                                       \
            hipLaunchKernelGGL((conv_chain<c, m, w, false>), grid, block, lds, s, x, y, a);           \
        }                                                                                              \
    } else
    PO2Q_CH(16, 2, false) PO2Q_CH(16, 4, false) PO2Q_CH(16, 8, false)
    PO2Q_CH(32, 2, false) PO2Q_CH(32, 4, false)
    PO2Q_CH(64, 2, true) PO2Q_CH(64, 4, true) PO2Q_CH(64, 2, false) PO2Q_CH(64, 4, false) {
        return false;
    }
#undef PO2Q_CH
        return true;
    };
    if (!launch(a)) {
        set_error("po2q: chain: no kernel for this shape");
        return PO2Q_ERR_INVALID;
    }
    he = hipGetLastError();
    if (he != hipSuccess) {
        set_error(std::string("po2q: chain launch: ") + hipGetErrorString(he));
        return PO2Q_ERR_HIP;
    }
#ifdef PO2Q_CHAIN_STAMPS
    if (getenv("PO2Q_STAMPS") && !a.stamps) {  // once more with the stamp buffer, summed per phase
        const size_t nst = (size_t)N * 8 * 8;
        if (hipMalloc(&a.stamps, nst * 4) == hipSuccess) {
            (void)hipMemsetAsync(a.stamps, 0, nst * 4, s);
            launch(a);
            std::vector<unsigned> h(nst);
            (void)hipStreamSynchronize(s);
            (void)hipMemcpy(h.data(), a.stamps, nst * 4, hipMemcpyDeviceToHost);
            (void)hipFree(a.stamps);
            double ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            for (int64_t b = 0; b < N; ++b)
                for (int w = 0; w < 8; ++w)
                    for (int i = 0; i < 8; ++i) ph[i] += h[((size_t)b * 8 + w) * 8 + i];
            fprintf(stderr, "[po2q chain stamps] C=%lld H=%lld W=%lld L=%d db=%d: cycles per layer per wave:", (long long)C,
                    (long long)H, (long long)W, n_layers, db ? 1 : 0);
            // per layer: top (loop top to the MFMAs: descriptor, epilogue constants; layer 0's also
            // the groups' address setup), mfma, bar1, epilogue, bar2; once: the prologue's x loads +
            // split (pro-split), residual loads (pro-res) and block barrier (pro-bar)
            const char* names[8] = {"top", "mfma", "bar1", "epilogue", "bar2", "pro-split", "pro-res", "pro-bar"};
            for (int i = 0; i < 8; ++i)
                fprintf(stderr, " %s %.0f", names[i], ph[i] / (double)(N * 8) / (i <= 4 ? n_layers : 1));
            fprintf(stderr, "\n");
        }
    }
#endif
    return PO2Q_OK;
}

}  // extern "C"
