// bf16x3 row-streaming conv, output channels split across the waves of a block:
// 3x3 / stride 1 / pad 1, C = 64, K = 64 (ResNet56 stage 3: 17 of its 56 qconvs).
//
// Same arithmetic as the other bf16x3 kernels (exact +-2^e bf16 weights x exact
// 3-way bf16 split of the fp32 activations, fp32 accumulation on
// v_mfma_f32_16x16x32_bf16; reference: QuantizedConv2d.forward,
// models/quantized_conv.py:32-38).  Stage 3 is MFMA-heavy (576 MACs per output
// element), so the layout is chosen for the matrix cores:
//
//   * a 4-wave block owns (image, strip of 32 output columns, segment of rows) and
//     marches down it one halo row at a time, like po2q_conv_rows.hip; wave w computes
//     output channels 16w .. 16w+15 for the whole strip;
//   * each wave's B fragments (3 tap rows x 2 channel chunks x 3 taps = 18 bf16x8)
//     stay in VGPRs for the kernel's lifetime -- no weight traffic in the loop;
//   * per halo row, wave w LDS-DMAs channels 16w .. 16w+15 of the strip (2 x 1 KiB)
//     plus 32 of the 128 halo-column values into a 2-slot raw ring, and splits
//     exactly what it loaded into the shared hi / mid / lo planes (double-buffered):
//     the DMA -> split dependency is wave-local (an exact vmcnt wait), and ONE block
//     barrier per row publishes the planes;
//   * every A fragment read from the planes feeds 3 MFMAs (the three output rows the
//     halo row touches); three accumulator slots rotate; loop unrolled by 6.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <type_traits>
#include <vector>

#include "po2q_internal.h"
#include "po2q_rows_dev.h"
#include "po2q_x3_dev.h"

namespace po2q {

namespace {

constexpr int kKC = 64;                        // input channels
constexpr int kKK = 64;                        // output channels = 4 waves x 16
constexpr int kKSW = 32;                       // strip width (2 pixel groups of 16)
constexpr int kKWC = kKSW + 2;                 // halo columns
constexpr int kKPlane = kKWC * kKC * 2;        // bytes per bf16 plane (128 B per pixel)
constexpr int kKPlanes = 3 * kKPlane;          // one plane buffer (hi, mid, lo)
constexpr int kKRawInt = kKC * kKSW * 4;       // raw interior [64][32] fp32 = 8 KiB
constexpr int kKRawSlot = kKRawInt + 4 * 256;  // + 4 waves x 64 halo dwords
constexpr int kKLds = 2 * kKPlanes + 2 * kKRawSlot;

// byte offset of (halo column hc, channel octet oct) in a plane: 128 B per pixel,
// octets XOR-swizzled by the column so 8 consecutive pixels of one octet spread over
// 8 bank quads (A-fragment reads 2-way at most)
__device__ __forceinline__ int k_addr(int hc, int oct) { return hc * 128 + ((oct ^ (hc & 7)) << 4); }

}  // namespace

struct RowsKArgs {
    int N, H, W, P, Q;
    int RB, nseg, nstrip, items;
    int remap;
};

__global__ __launch_bounds__(kThreads, 3) void conv_rowsk(const float* __restrict__ x, const uint4* __restrict__ wpk,
                                                          const float* __restrict__ scale_p,
                                                          const float* __restrict__ bias, float* __restrict__ y,
                                                          RowsKArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    unsigned char* planes = lds;                 // 2 buffers x 3 planes
    unsigned char* raw = lds + 2 * kKPlanes;     // 2 slots

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
    bf16x8 bw[3][6];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int ks = 0; ks < 6; ++ks)
            bw[r][ks] = __builtin_bit_cast(bf16x8, wpk[((r * 6 + ks) * 4 + wave) * 64 + lane]);
    const int kout = 16 * wave + (lane & 15);
    float bk = bias ? bias[kout] : 0.0f;
    const float scale = *scale_p;
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int ks = 0; ks < 6; ++ks) asm volatile("s_waitcnt vmcnt(0)" : "+v"(bw[r][ks]));
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(bk));

    // ---- DMA: wave w, instruction i: lane l -> channel 16w + 8i + (l >> 3), columns
    // 4*(l & 7) .. +3, landing at raw[c][col] (row-major, 128 B per channel); halo:
    // lanes 0..31 of wave w -> value v = 32w + lane: side v / 64, channel v % 64
    const int HW = a.H * a.W;
    const uint32_t cstride = (uint32_t)HW * 4u;
    const __amdgpu_buffer_rsrc_t rs = rows_rsrc(x + (int64_t)n * kKC * HW, kKC * HW * 4);
    const int cb = lane & 7;
    const int gq4 = q0 + 4 * cb;
    const bool qi_ok = gq4 < a.W;
    const uint32_t vi0 = (uint32_t)(16 * wave + (lane >> 3)) * cstride + (uint32_t)gq4 * 4u;
    const uint32_t soff1 = 8u * cstride;
    const int hv = 32 * wave + lane;
    const int hside = hv >> 6, hch = hv & 63;
    const int gqh = hside ? q0 + kKSW : q0 - 1;
    const bool qh_ok = lane < 32 && gqh >= 0 && gqh < a.W;
    const uint32_t vh0 = (uint32_t)hch * cstride + (uint32_t)gqh * 4u;
    const uint32_t raw_lds = (uint32_t)(uintptr_t)raw;

    // ---- split: lane -> (column sc, channel octet 2w + so), reading what this wave loaded
    const int sc = lane & 31, so = lane >> 5;
    const int oct = 2 * wave + so;
    const int rd0 = (8 * oct) * (kKSW * 4) + sc * 4;
    const int wa_i = k_addr(sc + 1, oct);
    const int wa_h = k_addr(hside ? kKWC - 1 : 0, hch >> 3) + (hch & 7) * 2;

    // ---- A fragment offsets: (group grp, chunk ch, tap s): pixel 16grp + p + s, octet 4ch + g
    int aoff[2][6];
    {
        const int p = lane & 15, g = lane >> 4;
#pragma unroll
        for (int grp = 0; grp < 2; ++grp)
#pragma unroll
            for (int ch = 0; ch < 2; ++ch)
#pragma unroll
                for (int s = 0; s < 3; ++s) aoff[grp][ch * 3 + s] = k_addr(16 * grp + p + s, 4 * ch + g);
    }

    auto load_row = [&](int sl, int j) __attribute__((always_inline)) {
        const int h = p0 - 1 + j;
        const bool hok = j < nrows && h >= 0 && h < a.H;
        const uint32_t roff = (uint32_t)(hok ? h : 0) * (uint32_t)a.W * 4u;
        const uint32_t vo = (hok && qi_ok) ? vi0 + roff : 0x7fffffffu;
        const uint32_t base = raw_lds + (uint32_t)(sl * kKRawSlot);
        rows_dma16(rs, vo, 0u, base + (uint32_t)(2 * wave) * 1024u);
        rows_dma16(rs, vo, soff1, base + (uint32_t)(2 * wave + 1) * 1024u);
        const uint32_t voh = (hok && qh_ok) ? vh0 + roff : 0x7fffffffu;
        rows_dma4(rs, voh, base + (uint32_t)kKRawInt + (uint32_t)wave * 256u);
    };
    constexpr int VMW = 7;  // 3 DMAs of the next row + 2 x 2 stores issued after a row's DMAs
    const int PQ = a.P * a.Q;
    const __amdgpu_buffer_rsrc_t ry = rows_rsrc(y + (int64_t)n * kKK * PQ, kKK * PQ * 4);

    floatx4 acc[3][2];
#pragma unroll
    for (int sl = 0; sl < 3; ++sl)
#pragma unroll
        for (int grp = 0; grp < 2; ++grp) acc[sl][grp] = floatx4{0.f, 0.f, 0.f, 0.f};

    auto step = [&](auto S_, int j) __attribute__((always_inline)) {
        constexpr int S6 = decltype(S_)::value;
        constexpr int S = S6 % 3;   // accumulator rotation
        constexpr int B2 = S6 % 2;  // raw slot and plane buffer
        unsigned char* pb = planes + B2 * kKPlanes;
        const unsigned char* rw = raw + B2 * kKRawSlot;
        rows_wait<VMW>();  // this wave's DMAs of row j have landed
        {
            uint32_t b8[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) b8[e] = *reinterpret_cast<const uint32_t*>(rw + rd0 + e * (kKSW * 4));
            uint4 hi, mid, lo;
            split3(b8, hi, mid, lo);
            *reinterpret_cast<uint4*>(pb + wa_i) = hi;
            *reinterpret_cast<uint4*>(pb + kKPlane + wa_i) = mid;
            *reinterpret_cast<uint4*>(pb + 2 * kKPlane + wa_i) = lo;
            if (lane < 32) {
                uint16_t h16, m16, l16;
                split1(*reinterpret_cast<const uint32_t*>(rw + kKRawInt + wave * 256 + 4 * lane), h16, m16, l16);
                *reinterpret_cast<uint16_t*>(pb + wa_h) = h16;
                *reinterpret_cast<uint16_t*>(pb + kKPlane + wa_h) = m16;
                *reinterpret_cast<uint16_t*>(pb + 2 * kKPlane + wa_h) = l16;
            }
        }
        // publish the planes: LDS writes done, then the block barrier (no memory fence:
        // the prefetches and stores in flight must not be waited for)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        // refill the raw slot this wave just split (its own data only)
        load_row(B2, j + 2);
        // MFMAs: halo row j feeds output halo-index j+1 (r=0), j (r=1), j-1 (r=2)
        constexpr int SL[3] = {(S + 1) % 3, S, (S + 2) % 3};
#pragma unroll
        for (int ks = 0; ks < 6; ++ks) {
            bf16x8 af[3][2];
#pragma unroll
            for (int pl = 0; pl < 3; ++pl)
#pragma unroll
                for (int grp = 0; grp < 2; ++grp)
                    af[pl][grp] = __builtin_bit_cast(
                        bf16x8, *reinterpret_cast<const uint4*>(pb + pl * kKPlane + aoff[grp][ks]));
#pragma unroll
            for (int rr = 0; rr < 3; ++rr)
#pragma unroll
                for (int pl = 0; pl < 3; ++pl)
#pragma unroll
                    for (int grp = 0; grp < 2; ++grp)
                        acc[SL[rr]][grp] =
                            __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[pl][grp], bw[rr][ks], acc[SL[rr]][grp], 0, 0, 0);
        }
        // output halo-index j-1 (row p0 + j - 2) is complete
        constexpr int D = (S + 2) % 3;
        const int o = p0 + j - 2;
        const bool orow = j >= 2 && o < p0 + rbe;
        const uint32_t yk = (uint32_t)kout * (uint32_t)PQ + (uint32_t)(orow ? o : 0) * a.Q;
#pragma unroll
        for (int grp = 0; grp < 2; ++grp) {
            const int q = q0 + 16 * grp + 4 * (lane >> 4);
            floatx4 v;
            v[0] = acc[D][grp][0] * scale + bk;
            v[1] = acc[D][grp][1] * scale + bk;
            v[2] = acc[D][grp][2] * scale + bk;
            v[3] = acc[D][grp][3] * scale + bk;
            rows_store(ry, (orow && q < a.Q) ? (yk + (uint32_t)q) * 4u : 0x7fffffffu, v);
            acc[D][grp] = floatx4{0.f, 0.f, 0.f, 0.f};
        }
    };

    {
        const floatx4 z = floatx4{0.f, 0.f, 0.f, 0.f};
        load_row(0, 0);
        rows_store(ry, 0x7fffffffu, z);
        rows_store(ry, 0x7fffffffu, z);
        load_row(1, 1);
        rows_store(ry, 0x7fffffffu, z);
        rows_store(ry, 0x7fffffffu, z);
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
    if (b.C != kKC || b.K != kKK || b.Q % 4 != 0) return;
    if ((int64_t)b.C * b.H * b.W * 4 >= (1LL << 31) || (int64_t)b.K * b.P * b.Q * 4 >= (1LL << 31)) return;
    ConvPlan p = b;
    p.kind = KIND_BF16X3_ROWS;
    p.vrx = 1;
    p.CC = 32;
    p.nchunks = 2;
    p.NT = 4;
    p.NJ = 2;
    p.TQ = kKSW;
    p.steps = 6;  // k-steps per tap row (2 chunks x 3 taps)
    p.kblocks = 1;
    p.taps = 9;
    p.PS = 0; p.MI = 0; p.pd = 2;
    p.dma_d0 = p.dma_nck = p.dma_ni = p.dma_nw = p.dma_waves = p.dma_ov = 0;
    p.HH = 0; p.WW = p.WWp = kKWC;
    p.SB = 2 * kKC;
    p.plane = kKPlane;
    p.lds_bytes = kKLds;
    p.packed_floats = (int64_t)3 * p.steps * p.NT * 64 * 4;
    p.tilesQ = (p.Q + kKSW - 1) / kKSW;
    const int slots = 256 * 3;  // blocks resident per chip (3 per CU: VGPR budget)
    std::vector<std::pair<double, int>> rbs;
    for (int rb = 4; rb <= p.P; ++rb) {
        const int nseg = (p.P + rb - 1) / rb;
        if (rb != (p.P + nseg - 1) / nseg) continue;
        const int64_t items = (int64_t)p.N * nseg * p.tilesQ;
        if (items > INT_MAX / 2) continue;
        rbs.push_back({(double)((items + slots - 1) / slots) * (rb + 2), rb});
    }
    std::sort(rbs.begin(), rbs.end());
    for (int i = 0; i < (int)rbs.size() && i < 3; ++i) {
        ConvPlan c = p;
        c.TP = rbs[i].second;
        c.tilesP = (p.P + c.TP - 1) / c.TP;
        const int64_t items = (int64_t)p.N * c.tilesP * c.tilesQ;
        c.blocks = (items + 7) / 8 * 8;
        out.push_back({0.9 + 0.001 * i, c});
    }
}

hipError_t launch_conv_rowsk(const ConvPlan& p, const float* x, const uint16_t* packed, const float* scale,
                             const float* bias, float* y, hipStream_t s) {
    RowsKArgs a;
    a.N = p.N; a.H = p.H; a.W = p.W; a.P = p.P; a.Q = p.Q;
    a.RB = p.TP; a.nseg = p.tilesP; a.nstrip = p.tilesQ;
    a.items = p.N * p.tilesP * p.tilesQ;
    a.remap = (p.blocks % 8 == 0) ? 1 : 0;
    hipLaunchKernelGGL(conv_rowsk, dim3((unsigned)p.blocks), dim3(kThreads), p.lds_bytes, s, x,
                       reinterpret_cast<const uint4*>(packed), scale, bias, y, a);
    return hipGetLastError();
}

}  // namespace po2q
