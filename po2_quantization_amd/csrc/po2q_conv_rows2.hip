// bf16x3 full-row-block conv for the stride-2 3x3 / pad-1 transition layers, C -> K = 2C with
// C = 16 or 32 (ResNet56 layer2.0.conv1 at 224x224 -> 112x112 and layer3.0.conv1 at 112x112
// -> 56x56; reference resnet.py:55-71, the first BasicBlock of a stage, each conv
// QuantizedConv2d.forward, quantized_conv.py:32-38).
//
// Same arithmetic as the other bf16x3 kernels (exact +-2^e bf16 weights x exact 3-way bf16
// split of the fp32 activations, fp32 accumulation on v_mfma_f32_16x16x32_bf16) and the
// same walk as conv_rowsf (po2q_conv_rowsf.hip): a block owns (image, segment of RB output
// rows) across the whole width, each input row is one cooperative whole-row LDS-DMA into a
// PD-slot ring, one s_barrier per input row, hand-counted vmcnt.  What stride 2 changes:
//   * wave w owns 16 output columns 16w .. 16w + 15, i.e. input columns 32w - 1 .. 32w + 31;
//     it splits them into an EVEN and an ODD sub-plane ([17 | 16 pixels][C] bf16), so the
//     tap-s pixel of output column p (input column 2p + s - 1) is E[p], O[p], E[p + 1] for
//     s = 0, 1, 2 -- 16 consecutive pixels of one sub-plane, conflict-free like stride 1;
//   * each input row feeds at most two output rows: an even-offset row adds tap row 1 to
//     output t, an odd-offset row adds tap row 2 to output t - 1 (which completes it) and
//     tap row 0 to output t: two accumulator slots rotate, output rows are stored every
//     other step (the steps between issue dropped stores, so the vmcnt count holds);
//   * both weights are quantized + packed by the block into LDS (fused staging): one launch;
//   * DS: the block's 1x1 / stride-2 / pad-0 projection shortcut (layer2.0.downsample.0 /
//     layer3.0.downsample.0, same C -> 2C) comes from the same x rows: its input pixel
//     (2t, 2p) is tap (1, 1) of output (t, p), so it is one more k-step of MFMAs on the
//     fragment the odd-offset row already holds, with its own quantized weight (own scale),
//     stored to a second output in the odd steps (dropped stores in the even ones).  x is
//     read once for both convs.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdint>
#include <cstdlib>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/po2q.h"
#include "po2q_epi.h"
#include "po2q_internal.h"
#include "po2q_quant_dev.h"
#include "po2q_rows_dev.h"
#include "po2q_x3_dev.h"

namespace po2q {

namespace {
constexpr int kR2EP = 17, kR2OP = 16;                          // even / odd sub-plane pixels
template <int CC> constexpr int kR2Plane = (kR2EP + kR2OP) * 2 * CC + 32;  // + zero slot
template <int CC> constexpr int kR2KS = CC == 16 ? 2 : 3;
}  // namespace

struct Rows2Args {
    int N, H, W, P, Q;
    int RB, nseg, items, remap;
    int rawslot;       // bytes per raw ring slot (>= ND x waves KiB: the DMAs past the row land in it)
    const float* ps;   // fused epilogue (EPI): y = act(y * ps[k] + pb[k]); either may be NULL
    const float* pb;
    int act;
    WQuant q;
    float* yds;        // DS: shortcut output [N, K, P, Q]; yds = Q(wds) * x[::2, ::2] (* psd[k] + pbd[k])
    WQuant qd;         // DS: the 1x1 weight [K, C, 1, 1]
    const float* psd;
    const float* pbd;
};

template <int CC, int PD, bool EPI, int NTS, int ND, bool DS = false>
__global__ __launch_bounds__(448, 2) void conv_rows2(const float* __restrict__ x, const float* __restrict__ bias,
                                                     float* __restrict__ y, Rows2Args a) {
    static_assert(CC == 16 || CC == 32, "C = 16 or 32");
    static_assert(PD == 2 || PD == 4, "ring slots: 4 % PD == 0 keeps every index static");
    constexpr int K = 2 * CC, NT = K / 16, KS = kR2KS<CC>, NF = 3 * KS * NT;
    constexpr int PL = kR2Plane<CC>, OBASE = kR2EP * 2 * CC, ZOFF = (kR2EP + kR2OP) * 2 * CC;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nw = (int)(blockDim.x >> 6);
    const int wv = wave;
    uint4* wl = reinterpret_cast<uint4*>(lds);                    // [NF][64] B fragments
    unsigned char* raw = lds + NF * 1024;                         // PD slots [C][W] fp32
    unsigned char* planes = lds + NF * 1024 + PD * a.rawslot;     // every wave's planes
    unsigned char* slab = planes + wave * (3 * PL);               // this wave's planes
    uint4* wld = reinterpret_cast<uint4*>(planes + nw * (3 * PL));  // DS: [NT][64]

    int blk = blockIdx.x;
    if (a.remap) blk = (blk & 7) * (int)(gridDim.x >> 3) + (blk >> 3);
    if (blk >= a.items) return;  // block-uniform
    const int seg = blk % a.nseg;
    const int n = blk / a.nseg;
    const int p0 = seg * a.RB;
    const int rbe = max(0, min(a.RB, a.P - p0));
    const int nrows = 2 * rbe + 1;  // input rows 2 p0 - 1 .. 2 (p0 + rbe) - 1
    const int nloop = nrows;
    const int q0 = 16 * wv;         // first output column of the wave

    // ---- DMA: lane l of this wave's instruction i -> float4 e = 64 (ndma w + i) + l of the
    // row's C x W/4 float4 (e past the row: out-of-range zeros into the slot's padding)
    const int HW = a.H * a.W;
    const __amdgpu_buffer_rsrc_t rs = rows_rsrc(x + (int64_t)n * CC * HW, CC * HW * 4);
    const int W4 = a.W >> 2;
    const uint32_t raw_lds = (uint32_t)(uintptr_t)raw;
    auto load_row = [&](int sl, int jn) __attribute__((always_inline)) {
        const int h = 2 * p0 - 1 + jn;
        const bool hok = jn < nrows && h >= 0 && h < a.H;
        const uint32_t roff = (uint32_t)(hok ? h : 0) * (uint32_t)a.W * 4u;
        const uint32_t base = raw_lds + (uint32_t)(sl * a.rawslot) + (uint32_t)(ND * wv) * 1024u;
#pragma unroll
        for (int i = 0; i < ND; ++i) {
            const int e = 64 * (ND * wv + i) + lane;
            const int c = e / W4, q = 4 * (e - c * W4);
            const uint32_t vo = (hok && c < CC) ? ((uint32_t)c * (uint32_t)HW + (uint32_t)q) * 4u + roff : 0x7fffffffu;
            rows_dma16<false>(rs, vo, 0u, base + i * 1024u);
        }
    };

    // ---- split tasks: (input column 2 q0 + t, channel octet o), t < 32; lane + 64 k
    constexpr int NTASK = 4 * CC / 64;  // 1 or 2 per lane
    int rd[NTASK], wa[NTASK];
    bool tok[NTASK];
#pragma unroll
    for (int k = 0; k < NTASK; ++k) {
        const int id = lane + 64 * k;
        const int t = id & 31, o = id >> 5;
        const int col = 2 * q0 + t;
        tok[k] = col < a.W;
        rd[k] = (o * 8) * (a.W * 4) + (tok[k] ? col : 0) * 4;
        // local index t + 1: odd t -> even pixel (t + 1) / 2, even t -> odd pixel t / 2
        wa[k] = (t & 1) ? x_addr<CC>((t + 1) >> 1, o) : OBASE + x_addr<CC>(t >> 1, o);
    }
    // left halo column 2 q0 - 1 -> even pixel 0 (lanes < C: one channel each)
    const int hcol = 2 * q0 - 1;
    const bool h_ok = lane < CC && hcol >= 0;
    const int rd_h = (lane % CC) * (a.W * 4) + (h_ok ? hcol : 0) * 4;
    const int wa_h = x_addr<CC>(0, (lane % CC) >> 3) + ((lane % CC) & 7) * 2;

    // ---- A fragment offsets per k-step (E[p], O[p], E[p+1] for taps 0, 1, 2)
    int aoff[KS];
    int ads;  // DS: the shortcut's own A fragment -- C = 16: k-step 0 with the tap-0 half read
              // from the zero slot, so a non-finite tap-0 pixel never meets the B fragment's
              // zero rows (inf * 0 = NaN where the 1x1 conv never reads that pixel)
    {
        const int p = lane & 15, g = lane >> 4;
        if constexpr (CC == 16) {
            aoff[0] = g < 2 ? x_addr<16>(p, g) : OBASE + x_addr<16>(p, g - 2);
            aoff[1] = g < 2 ? x_addr<16>(p + 1, g) : ZOFF;
            ads = g < 2 ? ZOFF : aoff[0];
        } else {
            aoff[0] = x_addr<32>(p, g);
            aoff[1] = OBASE + x_addr<32>(p, g);
            aoff[2] = x_addr<32>(p + 1, g);
            ads = aoff[1];
        }
    }

    const int PQ = a.P * a.Q;
    const __amdgpu_buffer_rsrc_t ry = rows_rsrc(y + (int64_t)n * K * PQ, K * PQ * 4);
    constexpr int ST = DS ? 2 * NT : NT;  // stores per step (every step; the idle output's are dropped)
    const __amdgpu_buffer_rsrc_t ryd = rows_rsrc(DS ? a.yds + (int64_t)n * K * PQ : y, DS ? K * PQ * 4 : 4);
    float scaled = 1.0f;
    bool find = true;
    float epsd[NT], epbd[NT];
    floatx4 accd[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) accd[nt] = floatx4{0.f, 0.f, 0.f, 0.f};

    float scale = 1.0f;
    bool fin = true;
    float bk[NT], eps_[NT], epb_[NT];
    floatx4 acc[2][NT];
#pragma unroll
    for (int sl = 0; sl < 2; ++sl)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[sl][nt] = floatx4{0.f, 0.f, 0.f, 0.f};

    // MFMAs of the split row with tap row rr into accumulator slot SLOT
    auto mfmas = [&](auto RR_, auto SLOT_) __attribute__((always_inline)) {
        constexpr int RR = decltype(RR_)::value, SLOT = decltype(SLOT_)::value;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            bf16x8 af[3];
#pragma unroll
            for (int pl = 0; pl < 3; ++pl)
                af[pl] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(slab + pl * PL + aoff[ks]));
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
                const bf16x8 b = __builtin_bit_cast(bf16x8, wl[((RR * KS + ks) * NT + nt) * 64 + lane]);
#pragma unroll
                for (int pl = 0; pl < 3; ++pl)
                    acc[SLOT][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[pl], b, acc[SLOT][nt], 0, 0, 0);
            }
        }
    };
    // store output row p0 + o from slot SLOT (dropped when `valid` is false), then zero it
    auto store_row = [&](auto SLOT_, int o, bool valid) __attribute__((always_inline)) {
        constexpr int SLOT = decltype(SLOT_)::value;
        const bool orow = valid && o >= 0 && o < rbe;
        const int g = lane >> 4;
        const int q = q0 + 4 * g;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
            const int k = 16 * nt + (lane & 15);
            floatx4 v;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float t = acc[SLOT][nt][e] * scale + bk[nt];
                if constexpr (EPI) t = epi_act(t * eps_[nt] + epb_[nt], a.act);
                v[e] = t;
            }
            const uint32_t yo = (uint32_t)k * (uint32_t)PQ + (uint32_t)(orow ? p0 + o : 0) * a.Q + (uint32_t)q;
            rows_store<(NTS & 1) != 0>(ry, (orow && q < a.Q) ? yo * 4u : 0x7fffffffu, v);
            if (valid) acc[SLOT][nt] = floatx4{0.f, 0.f, 0.f, 0.f};
        }
    };

    // DS: the shortcut of output row t (local) from the odd-offset row's tap-1 fragment, stored
    // when `valid` (else NT dropped stores keep the count)
    auto ds_row = [&](int t, bool valid) __attribute__((always_inline)) {
        if (valid) {
            bf16x8 af[3];
#pragma unroll
            for (int pl = 0; pl < 3; ++pl)
                af[pl] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(slab + pl * PL + ads));
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
                const bf16x8 b = __builtin_bit_cast(bf16x8, wld[nt * 64 + lane]);
#pragma unroll
                for (int pl = 0; pl < 3; ++pl)
                    accd[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[pl], b, accd[nt], 0, 0, 0);
            }
        }
        const bool orow = valid && t >= 0 && t < rbe;
        const int q = q0 + 4 * (lane >> 4);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
            const int k = 16 * nt + (lane & 15);
            floatx4 v;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float u = accd[nt][e] * scaled;
                if constexpr (EPI) u = u * epsd[nt] + epbd[nt];
                v[e] = u;
            }
            const uint32_t yo = (uint32_t)k * (uint32_t)PQ + (uint32_t)(orow ? p0 + t : 0) * a.Q + (uint32_t)q;
            rows_store<(NTS & 1) != 0>(ryd, (orow && q < a.Q) ? yo * 4u : 0x7fffffffu, v);
            if (valid) accd[nt] = floatx4{0.f, 0.f, 0.f, 0.f};
        }
    };

    // vm ops after this wave's DMAs of row j (issued in step j - PD + 1, after its barrier)
    // until the wait of step j: that step's ST stores, then ND DMAs + ST stores per step
    constexpr int VMW = ST + (PD - 2) * (ND + ST);
    auto step = [&](auto S_, int j) __attribute__((always_inline)) {
        constexpr int S4 = decltype(S_)::value;  // j % 4
        constexpr int RS = S4 % PD;
        rows_wait<VMW>();
        __builtin_amdgcn_s_barrier();  // every wave's DMAs of row j landed; row j - 1 is split
        load_row((S4 + PD - 1) % PD, j - 1 + PD);
        // split input row j: the wave's 32 columns (+ the left halo column)
        {
            const unsigned char* rw = raw + RS * a.rawslot;
#pragma unroll
            for (int k = 0; k < NTASK; ++k) {
                uint32_t b8[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) b8[e] = *reinterpret_cast<const uint32_t*>(rw + rd[k] + e * (a.W * 4));
                if (!tok[k]) {
#pragma unroll
                    for (int e = 0; e < 8; ++e) b8[e] = 0u;
                }
                uint4 hi, mid, lo;
                split3(b8, hi, mid, lo);
                *reinterpret_cast<uint4*>(slab + wa[k]) = hi;
                *reinterpret_cast<uint4*>(slab + PL + wa[k]) = mid;
                *reinterpret_cast<uint4*>(slab + 2 * PL + wa[k]) = lo;
            }
            if (lane < CC) {
                uint32_t hb = *reinterpret_cast<const uint32_t*>(rw + rd_h);
                hb = h_ok ? hb : 0u;
                uint16_t h16, m16, l16;
                split1(hb, h16, m16, l16);
                *reinterpret_cast<uint16_t*>(slab + wa_h) = h16;
                *reinterpret_cast<uint16_t*>(slab + PL + wa_h) = m16;
                *reinterpret_cast<uint16_t*>(slab + 2 * PL + wa_h) = l16;
            }
        }
        // input row j: even j = 2t -> tap row 0 into output t, tap row 2 into output t - 1
        // (complete: stored); odd j = 2t + 1 -> tap row 1 into output t
        const int t = j >> 1;
        if constexpr ((S4 & 1) == 0) {
            constexpr int CUR = (S4 >> 1) & 1, PREV = CUR ^ 1;
            mfmas(std::integral_constant<int, 2>{}, std::integral_constant<int, PREV>{});
            mfmas(std::integral_constant<int, 0>{}, std::integral_constant<int, CUR>{});
            store_row(std::integral_constant<int, PREV>{}, t - 1, true);
            if constexpr (DS) ds_row(t, false);  // dropped: keeps the count
        } else {
            constexpr int CUR = (S4 >> 1) & 1;
            mfmas(std::integral_constant<int, 1>{}, std::integral_constant<int, CUR>{});
            store_row(std::integral_constant<int, CUR>{}, t, false);  // dropped: keeps the count
            if constexpr (DS) ds_row(t, true);   // input row 2 (p0 + t): the shortcut of output t
        }
    };

    {
        const floatx4 z = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int r = 0; r < PD - 1; ++r) {
            load_row(r, r);
#pragma unroll
            for (int i = 0; i < ST; ++i) rows_store<(NTS & 1) != 0>(ry, 0x7fffffffu, z);
        }
    }
    // ---- weights: quantize + pack into LDS while those DMAs fly (scratch: wave 0's planes)
    {
        unsigned* red = reinterpret_cast<unsigned*>(planes);
        unsigned* thr = red + 16;
        scale = wq_prologue(a.q, thr, red, nw, fin);
        __syncthreads();  // every wave's scratch reads done before wl (disjoint) -- and thr stays
        wq_pack_rows_lds<CC>(a.q, K, CC, NT, KS, scale, fin, thr, wl, NF);
        if constexpr (DS) {
            __syncthreads();  // thr / red reads of the 3x3 weight done
            scaled = wq_prologue(a.qd, thr, red, nw, find);
            for (int e = tid; e < NT * 64; e += blockDim.x) {
                // B fragment of k-step KDS: rows k = 8 g .. 8 g + 7 (g = lane >> 4) are tap 1's
                // channels (C = 32: c = 8 g + i; C = 16: g >= 2, c = 8 (g & 1) + i; else zero)
                const int l = e & 63, nt = e >> 6, g = l >> 4, k = 16 * nt + (l & 15);
                const bool ok = CC == 32 || g >= 2;
                const int c0 = CC == 32 ? 8 * g : 8 * (g & 1);
                uint32_t h[8];
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    h[i] = ok ? pack_one(a.qd.w[k * CC + c0 + i], scaled, find, a.qd.mode, a.qd.lo, a.qd.hi, thr) : 0u;
                wld[e] = make_uint4(h[0] | (h[1] << 16), h[2] | (h[3] << 16), h[4] | (h[5] << 16), h[6] | (h[7] << 16));
            }
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
                const int k = 16 * nt + (lane & 15);
                epsd[nt] = (EPI && a.psd) ? a.psd[k] : 1.0f;
                epbd[nt] = (EPI && a.pbd) ? a.pbd[k] : 0.0f;
            }
        }
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
            const int k = 16 * nt + (lane & 15);
            bk[nt] = bias ? bias[k] : 0.0f;
            eps_[nt] = (EPI && a.ps) ? a.ps[k] : 1.0f;
            epb_[nt] = (EPI && a.pb) ? a.pb[k] : 0.0f;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) asm volatile("" : "+v"(bk[nt]), "+v"(eps_[nt]), "+v"(epb_[nt]));
        if constexpr (DS) {
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) asm volatile("" : "+v"(epsd[nt]), "+v"(epbd[nt]));
        }
        __syncthreads();  // wl complete, scratch free
        if (lane < 3) *reinterpret_cast<uint4*>(slab + lane * PL + ZOFF) = make_uint4(0u, 0u, 0u, 0u);
    }
    // the last output row completes (and is stored) at step nrows - 1 = 2 rbe
    for (int j = 0; j < nloop; j += 4) {
        step(std::integral_constant<int, 0>{}, j);
        step(std::integral_constant<int, 1>{}, j + 1);
        if (j + 2 >= nloop) break;
        step(std::integral_constant<int, 2>{}, j + 2);
        step(std::integral_constant<int, 3>{}, j + 3);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // trailing DMAs land before the wave ends
}

// ------------------------------------------------------------------ planning --
static size_t rows2_lds(int C, int waves, int pd, int rawslot) {
    const int nf = 3 * (C == 16 ? 2 : 3) * (2 * C / 16);
    const int plane = (kR2EP + kR2OP) * 2 * C + 32;
    return (size_t)nf * 1024 + (size_t)pd * rawslot + (size_t)waves * 3 * plane;
}

void rows2_candidates(const ConvPlan& b, int mode, int bits, int fsr, std::vector<PlanCand>& out) {
    if (mode == 0 || b.groups != 1) return;
    if (bits < 1 || bits > 16) return;
    const long lo = (long)fsr - (1L << (bits - 1)), hi = (long)fsr - 1;
    if (lo < -126 || hi > 127) return;  // +-2^e must be a normal bf16
    if (b.R != 3 || b.S != 3 || b.sh != 2 || b.sw != 2 || b.ph != 1 || b.pw != 1 || b.dh != 1 || b.dw != 1) return;
    // the instantiated shapes: ResNet56 layer2.0.conv1 (16 -> 32) and layer3.0.conv1 (32 -> 64)
    if (!((b.C == 16 && b.K == 32) || (b.C == 32 && b.K == 64))) return;
    if (b.W % 4 != 0 || b.Q % 4 != 0) return;
    const int waves = (b.Q + 15) / 16;
    if (waves < 1 || waves > 7 || 32 * waves < b.W) return;  // the waves' input strips cover the row
    if ((int64_t)b.C * b.H * b.W * 4 >= (1LL << 31) || (int64_t)b.K * b.P * b.Q * 4 >= (1LL << 31)) return;
    if ((int64_t)b.K * b.C * 9 > 65536) return;  // fused staging: every block reads the weight
    ConvPlan p = b;
    p.kind = KIND_BF16X3_ROWS;
    p.vrx = 5;  // stride-2 full-row blocks
    p.CC = b.C; p.NT = b.K / 16; p.NJ = 1; p.TQ = 16 * waves;
    p.steps = b.C == 16 ? 2 : 3; p.nchunks = 1; p.kblocks = 1; p.taps = 9;
    p.PS = 0; p.MI = 0; p.fp = 1;
    p.dma_d0 = p.dma_nck = p.dma_ni = p.dma_nw = p.dma_waves = p.dma_ov = 0;
    p.HH = 0; p.WW = p.WWp = 33;
    p.SB = 2 * b.C;
    p.plane = (kR2EP + kR2OP) * 2 * b.C + 32;
    p.packed_floats = (int64_t)3 * p.steps * p.NT * 64 * 4;
    p.tilesQ = 1;
    const int total4 = b.C * b.W / 4;                      // float4 per input row
    const int ndma = (total4 + 64 * waves - 1) / (64 * waves);
    if (ndma < 1 || ndma > (b.C == 16 ? 2 : 4)) return;  // instantiated DMA counts per wave
    const int rawslot = std::max(b.C * b.W * 4, ndma * waves * 1024);
    p.dma_ni = ndma;
    p.dma_nck = rawslot;
    for (int pd : {2, 4}) {
        if (b.C == 32 && pd != 2) continue;  // C = 32: one block per CU already at pd 2 (LDS)
        ConvPlan q = p;
        q.pd = pd;
        q.lds_bytes = rows2_lds(b.C, waves, pd, rawslot);
        const int per_cu = std::min(2, (int)(160 * 1024 / q.lds_bytes));
        if (per_cu < 1) continue;
        // segments: every CU busy with per_cu blocks, one extra input row per segment
        int nseg = std::max(1, (256 * per_cu + b.N - 1) / b.N);
        nseg = std::min(nseg, std::max(1, b.P / 4));
        int prev = -1;
        for (int f : {1, 2}) {
            ConvPlan c = q;
            const int ns = std::min(nseg * f, std::max(1, b.P / 4));
            if (ns == prev) break;
            prev = ns;
            c.TP = (b.P + ns - 1) / ns;
            c.tilesP = (b.P + c.TP - 1) / c.TP;
            c.blocks = ((int64_t)b.N * c.tilesP + 7) / 8 * 8;
            for (int nts : {0, 1}) {
                if (b.C == 32 && nts) continue;
                c.nts = nts;
                out.push_back({0.885 + 0.001 * (f - 1) + 0.002 * nts + 0.001 * (pd - 2), c});
            }
        }
    }
}

template <int CC, int PD, bool EPI, int NTS, int ND>
static hipError_t launch_rows2_nd(const ConvPlan& p, const Rows2Args& a, const float* x, const float* bias, float* y,
                                  hipStream_t s) {
    if (p.PS != 0) return hipErrorInvalidValue;
    if (a.yds)
        hipLaunchKernelGGL((conv_rows2<CC, PD, EPI, NTS, ND, true>), dim3((unsigned)p.blocks), dim3(64 * (p.TQ / 16)),
                           p.lds_bytes + (size_t)(2 * CC / 16) * 1024, s, x, bias, y, a);
    else
        hipLaunchKernelGGL((conv_rows2<CC, PD, EPI, NTS, ND>), dim3((unsigned)p.blocks), dim3(64 * (p.TQ / 16)),
                           p.lds_bytes, s, x, bias, y, a);
    return hipGetLastError();
}

template <int CC, int PD, bool EPI, int NTS>
static hipError_t launch_rows2_t(const ConvPlan& p, const Rows2Args& a, const float* x, const float* bias, float* y,
                                 hipStream_t s) {
    switch (p.dma_ni) {
        case 1: return launch_rows2_nd<CC, PD, EPI, NTS, 1>(p, a, x, bias, y, s);
        case 2: return launch_rows2_nd<CC, PD, EPI, NTS, 2>(p, a, x, bias, y, s);
        case 3: if constexpr (CC == 32) return launch_rows2_nd<CC, PD, EPI, NTS, 3>(p, a, x, bias, y, s); break;
        case 4: if constexpr (CC == 32) return launch_rows2_nd<CC, PD, EPI, NTS, 4>(p, a, x, bias, y, s); break;
        default: break;
    }
    return hipErrorInvalidValue;
}

hipError_t launch_conv_rows2(const ConvPlan& p, const float* x, const float* bias, float* y, hipStream_t s,
                             const float* ps, const float* pb, int act, bool epi, const WQuant& q, float* yds,
                             const WQuant& qd, const float* psd, const float* pbd) {
    if (p.kind != KIND_BF16X3_ROWS || p.vrx != 5 || !q.w || !((p.C == 16 && p.K == 32) || (p.C == 32 && p.K == 64)))
        return hipErrorInvalidValue;
    if (yds && (!qd.w || p.lds_bytes + (size_t)(p.K / 16) * 1024 > 160 * 1024)) return hipErrorInvalidValue;
    Rows2Args a;
    a.N = p.N; a.H = p.H; a.W = p.W; a.P = p.P; a.Q = p.Q;
    a.RB = p.TP;
    a.nseg = p.tilesP;
    a.items = p.N * a.nseg;
    a.remap = (p.blocks % 8 == 0) ? 1 : 0;
    a.rawslot = p.dma_nck;
    a.ps = ps; a.pb = pb; a.act = act;
    a.q = q;
    a.yds = yds; a.qd = qd; a.psd = psd; a.pbd = pbd;
#define PO2Q_R2(d, e, nt) \
    if (p.C == 16 && p.pd == d && epi == e && p.nts == nt) return launch_rows2_t<16, d, e, nt>(p, a, x, bias, y, s);
    PO2Q_R2(2, false, 0) PO2Q_R2(2, false, 1) PO2Q_R2(4, false, 0) PO2Q_R2(4, false, 1)
    PO2Q_R2(2, true, 0) PO2Q_R2(2, true, 1) PO2Q_R2(4, true, 0) PO2Q_R2(4, true, 1)
#undef PO2Q_R2
    if (p.C == 32 && p.pd == 2 && p.nts == 0)
        return epi ? launch_rows2_t<32, 2, true, 0>(p, a, x, bias, y, s) : launch_rows2_t<32, 2, false, 0>(p, a, x, bias, y, s);
    return hipErrorInvalidValue;
}

}  // namespace po2q

// ------------------------------------------------------------------ C ABI --
namespace {

// The stride-2 plan for the fused conv + shortcut: the plan the sweeps measured fastest
// (profiles/r02_stage_s2*_sweep.jsonl: C = 16 ring depth 4, C = 32 depth 2; whole-image
// segments at bs >= 256), else the first stride-2 candidate.
bool s2ds_plan(po2q::ConvPlan& p, int64_t N, int64_t C, int64_t H, int64_t W, int bits, int fsr, int mode) {
    if (N <= 0 || H <= 0 || W <= 0 || !((C == 16) || (C == 32))) return false;
    if (mode != PO2Q_MODE_PO2 && mode != PO2Q_MODE_PO2_PLUS) return false;
    std::vector<po2q::ConvPlan> cands;
    if (!po2q::plan_candidates(cands, N, C, H, W, 2 * C, 3, 3, 2, 2, 1, 1, 1, 1, 1, mode, bits, fsr, PO2Q_PREC_BF16X3))
        return false;
    const int want = C == 16 ? 4 : 2;
    int pick = -1;
    auto score = [&](const po2q::ConvPlan& c) { return c.pd == want ? 1 : 0; };
    for (int i = 0; i < (int)cands.size(); ++i) {
        const po2q::ConvPlan& c = cands[i];
        if (c.kind != po2q::KIND_BF16X3_ROWS || c.vrx != 5 || c.nts != 0) continue;
        if (c.lds_bytes + (size_t)(2 * C / 16) * 1024 > 160 * 1024) continue;
        if (pick < 0 || score(c) > score(cands[pick])) pick = i;
    }
    if (pick < 0) return false;
    p = cands[pick];
    return true;
}

}  // namespace

int po2q_qconv2d_s2ds_supported(int64_t N, int64_t C, int64_t H, int64_t W, int bits, int fsr, int mode) {
    // advisory: the fused transition is the faster path on wide rows (ResNet56 @224: W = 224 /
    // 112), slower on CIFAR-size rows (@32, W = 32 / 16: 2.17-2.20 vs 2.02-2.08 ms per forward,
    // profiles/r02_ab_s2ds_small.txt); po2q_qconv2d_s2ds_f32 itself takes both
    if (W < 96) return 0;
    po2q::ConvPlan p;
    return s2ds_plan(p, N, C, H, W, bits, fsr, mode) ? 1 : 0;
}

int po2q_qconv2d_s2ds_f32(const float* x, const float* w, const float* wds, float* y, float* yds, int64_t N,
                          int64_t C, int64_t H, int64_t W, int bits, int fsr, int mode, const float* post_scale,
                          const float* post_shift, int act, const float* post_scale_ds, const float* post_shift_ds,
                          void* stream) {
    if (!x || !w || !wds || !y || !yds) {
        po2q::set_error("po2q: s2ds: null pointer");
        return PO2Q_ERR_INVALID;
    }
    if (bits < 1 || bits > 16) {
        po2q::set_error("po2q: bits must be in [1, 16]");
        return PO2Q_ERR_INVALID;
    }
    if (act < PO2Q_ACT_NONE || act > PO2Q_ACT_SILU) {
        po2q::set_error("po2q: unknown activation");
        return PO2Q_ERR_INVALID;
    }
    if (y == yds || x == y || x == yds) {
        po2q::set_error("po2q: s2ds: y, yds and x must not alias");
        return PO2Q_ERR_INVALID;
    }
    po2q::ConvPlan p;
    if (!s2ds_plan(p, N, C, H, W, bits, fsr, mode)) {
        po2q::set_error("po2q: s2ds: 3x3 stride-2 C -> 2C with C = 16 or 32 and a po2 / po2+ weight only");
        return PO2Q_ERR_UNSUPPORTED;
    }
    po2q::WQuant q, qd;
    q.w = w;
    q.n = (int)(2 * C * C * 9);
    q.lo = fsr - (1 << (bits - 1));
    q.hi = fsr - 1;
    q.mode = mode - 1;
    qd = q;
    qd.w = wds;
    qd.n = (int)(2 * C * C);
    const bool epi = post_scale || post_shift || act != PO2Q_ACT_NONE || post_scale_ds || post_shift_ds;
    const hipError_t e = po2q::launch_conv_rows2(p, x, nullptr, y, reinterpret_cast<hipStream_t>(stream), post_scale,
                                                 post_shift, act, epi, q, yds, qd, post_scale_ds, post_shift_ds);
    if (e != hipSuccess) {
        po2q::set_error(std::string("po2q: s2ds launch: ") + hipGetErrorString(e));
        return PO2Q_ERR_HIP;
    }
    return PO2Q_OK;
}

