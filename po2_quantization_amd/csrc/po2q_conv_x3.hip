// bf16x3 split-exact implicit-GEMM convolution for gfx950 (the PO2 hot path).
//
// Reference: QuantizedConv2d.forward (models/quantized_conv.py:32-38) =
//   F.conv2d(x, Q(w), bias, stride, padding, dilation) with Q the PO2 / PO2+
//   quantizer (utils/quantizers.py:19-52), NCHW fp32 in and out.
//
// Why bf16 MFMA gives fp32 results here:
//   * Q(w) = (2^e * sign(w)) * scale, so W' = Q(w) / scale = +-2^e (or 0) is
//     EXACT in bf16 for every exponent the quantizer can produce (e >= -126).
//   * Every fp32 activation splits exactly into three bf16 terms by bit
//     truncation: hi = x & 0xffff0000, mid = (x - hi) & 0xffff0000,
//     lo = x - hi - mid (each remainder carries <= 16, then <= 8 significant bits).
//   * v_mfma_f32_16x16x32_bf16 forms the products W' * {hi, mid, lo} exactly and
//     accumulates in fp32; y = scale * acc (+ bias).  The only roundings are the
//     fp32 accumulations -- the same class of error as the reference's fp32 conv
//     (parity contract: max|y - y_ref| <= 1e-5 max|y_ref|, tests/_util.py).
//   Three bf16 MFMAs cost 3/16 of one fp32 MFMA (MI355X: 2.5 PF bf16 vs 157 TF
//   fp32), which moves every ResNet56 layer from the fp32 matrix roof to HBM.
//
// Kernel structure (one 256-thread block = 4 waves per output tile):
//   tile = TP x TQ output pixels of one image x (16*NT) output channels;
//   per input-channel chunk of CC channels:
//     x halo tile  HBM fp32 NCHW -> split hi/mid/lo -> LDS, three planes laid out
//                  [halo pixel][CC] bf16 (pixel stride SB = 2*CC bytes; CC = 32
//                  XOR-swizzles the channel octet with pixel bits 1..2), so an
//                  MFMA A-fragment (16 pixels x 8 consecutive k) is one
//                  conflict-free ds_read_b128 per lane (tools/lds_banks.py);
//     weights      pre-packed B fragments (po2q_quant.hip) -> LDS, 1 KiB per
//                  (k-step, 16-channel tile);
//   GEMM: M = pixels (NJ groups of 16 per wave), N = output channels (NT tiles),
//         k = (tap, channel) tap-major, 32 per MFMA k-step; padded taps read a
//         zero 16-byte slot (never a real pixel: 0 * inf must not appear).
//   Epilogue: D[pixel][channel] -> lane holds 4 consecutive pixels of one
//   channel -> one float4 store per (group, tile) into NCHW y.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "po2q_internal.h"
#include "po2q_x3_dev.h"

namespace po2q {


struct X3Args {
    int N, C, H, W, K, P, Q, sh, sw, ph, pw, dh, dw, R, S;
    int TP, TQ, tilesP, tilesQ, kblocks, nchunks, HH, WW, ksteps, taps;
    int plane;     // bytes per split plane (halo pixels * SB + 16 zero bytes)
    int w_off;     // LDS byte offset of the weight fragments
    int tap_off;   // LDS byte offset of the tap offset table
    int bias_off;  // LDS byte offset of the bias (kblocks * 16 * NT floats, 0 past K)
    int vec;       // float4 epilogue allowed (Q % 4 == 0 && TQ % 4 == 0)
    int remap;     // XCD-aware block remap (nblocks % 8 == 0)
    int nblocks;
    int dbg;       // diagnostics only (PO2Q_X3_DEBUG): 1 no MFMA, 2 no split, 4 no x loads, 8 no stores
};

constexpr int kXI = 3;  // max x-staging items (pixel x channel octet) per thread per work item
constexpr int kWI = 5;  // max weight fragments (uint4) per thread per chunk

// Persistent, software-pipelined: each block walks work items (tile, chunk) =
// blockIdx.x + i*gridDim.x tiles x nchunks chunks.  The NEXT item's x halo
// (fp32, straight to registers) and weight fragments are loaded right after
// the current item is in LDS, so HBM latency hides behind the MFMA work and
// the epilogue stores of the current item.
//   x loads: raw buffer loads, one 32-bit voffset per staged item and the
//   channel stride in the SGPR soffset (8 loads, zero address VALU); halo
//   pixels outside the image and channels >= C get an out-of-range offset, so
//   the hardware bounds check returns the zero padding.
//   KS > 0: compile-time k-steps per chunk (tap offsets live in registers).
template <int CC, int NT, int NJ, int KS, bool MC, int PD>
__global__ __launch_bounds__(kThreads, 2) void conv_bf16x3(const float* __restrict__ x,
                                                           const uint4* __restrict__ wpk,
                                                           const float* __restrict__ scale_p,
                                                           const float* __restrict__ bias, float* __restrict__ y,
                                                           X3Args a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    constexpr int OCT = CC / 8;  // channel octets per tap
    constexpr int KSR = KS ? KS : 1;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int T = a.nblocks;     // total tiles (N * kblocks * tilesP * tilesQ)
    const int npix = a.TP * a.TQ;
    const int hw_halo = a.HH * a.WW;
    const int zero_off = hw_halo * (2 * CC);  // 16 zero bytes after the halo pixels of each plane
    const int items = hw_halo * OCT;
    const int ksteps = KS ? KS : a.ksteps;
    const int kfr = ksteps * NT * 64;         // weight fragments (uint4) per chunk
    const int64_t HWi = (int64_t)a.H * a.W;
    const uint32_t cstride = (uint32_t)HWi * 4u;  // channel stride, bytes (planner: < 2^28)
    int v = blockIdx.x;
    if (v >= T) return;
    const int o = lane >> 4;

    int* tapt = reinterpret_cast<int*>(lds + a.tap_off);
    if (!KS && tid < a.taps) {
        const int r = tid / a.S, s = tid - (tid / a.S) * a.S;
        tapt[tid] = r * a.dh * a.WW + s * a.dw;
    }
    if (tid < 3) *reinterpret_cast<uint4*>(lds + tid * a.plane + zero_off) = make_uint4(0u, 0u, 0u, 0u);
    float* bias_l = reinterpret_cast<float*>(lds + a.bias_off);
    for (int k = tid; k < a.kblocks * 16 * NT; k += kThreads) bias_l[k] = (bias && k < a.K) ? bias[k] : 0.0f;

    // halo pixel of this lane's pixel in each group (tile-linear, row-major);
    // epilogue position of its 4-pixel run
    int hp0[NJ], ep[NJ];
#pragma unroll
    for (int g = 0; g < NJ; ++g) {
        int slot = (wave * NJ + g) * 16 + (lane & 15);
        if (slot >= npix) slot = 0;
        const int pl = slot / a.TQ, ql = slot - (slot / a.TQ) * a.TQ;
        hp0[g] = pl * a.sh * a.WW + ql * a.sw;
        const int i0 = (wave * NJ + g) * 16 + 4 * o;
        ep[g] = (i0 < npix) ? (((i0 / a.TQ) << 16) | (i0 - (i0 / a.TQ) * a.TQ)) : -1;
    }
    // per-lane tap offsets for compile-time k-steps: pixel offset, channel octet, pad flag
    int tpx[KSR], tco[KSR];
    unsigned padm = 0;
    if constexpr (KS > 0) {
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const int oi = ks * 4 + o;
            const int t = oi / OCT;
            tco[ks] = oi % OCT;
            const int r = t / a.S, s = t - (t / a.S) * a.S;
            tpx[ks] = r * a.dh * a.WW + s * a.dw;
            if (t >= a.taps) padm |= 1u << ks;
        }
    }
    // staging descriptors: this thread's (halo row, halo col, channel octet) per item
    uint32_t pk[kXI];
#pragma unroll
    for (int r = 0; r < kXI; ++r) {
        const int it = tid + r * kThreads;
        const int oc = it / hw_halo;
        const int hp = it - oc * hw_halo;
        const int hh = hp / a.WW, ww = hp - (hp / a.WW) * a.WW;
        pk[r] = (it < items) ? (0x80000000u | ((uint32_t)hh << 20) | ((uint32_t)ww << 8) | (uint32_t)oc) : 0u;
    }

    uint32_t xa[kXI][8], xb[PD == 2 ? kXI : 1][PD == 2 ? 8 : 1];
    // weight staging registers (multi-chunk): five named uint4s, not an array -- an
    // array here was left dynamically indexed and lived in scratch memory
    static_assert(kWI == 5, "weight staging is written out for kWI == 5");
    uint4 wr0, wr1, wr2, wr3, wr4;
#define PO2Q_W_ALL(OP) OP(0, wr0) OP(1, wr1) OP(2, wr2) OP(3, wr3) OP(4, wr4)

    auto load_x = [&](uint32_t (&xr)[kXI][8], const TileCoord& tc, int chunk) __attribute__((always_inline)) {
        const int h0 = tc.p0 * a.sh - a.ph, w0 = tc.q0 * a.sw - a.pw;
        const float* base = x + ((int64_t)tc.n * a.C + chunk * CC) * HWi;
        const int64_t rem = (int64_t)(a.C - chunk * CC) * HWi * 4;
        const int nrec = (int)(rem > 0x7fffffffLL ? 0x7fffffffLL : rem);
        const uintptr_t bp = reinterpret_cast<uintptr_t>(base);
        const uint32_t blo = __builtin_amdgcn_readfirstlane((uint32_t)bp);
        const uint32_t bhi = __builtin_amdgcn_readfirstlane((uint32_t)(bp >> 32));
        const void* bu = reinterpret_cast<const void*>(((uintptr_t)bhi << 32) | blo);
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(bu), (short)0,
                                                                           __builtin_amdgcn_readfirstlane(nrec),
                                                                           0x00020000);
#pragma unroll
        for (int r = 0; r < kXI; ++r) {
            const uint32_t d = pk[r];
            const int hh = (int)((d >> 20) & 0x7ffu), ww = (int)((d >> 8) & 0xfffu), oc = (int)(d & 0xffu);
            const int h = h0 + hh, w = w0 + ww;
            const bool ok = (d >> 31) && ((unsigned)h < (unsigned)a.H) && ((unsigned)w < (unsigned)a.W) &&
                            !(kDbg(a) & 4);
            const uint32_t vo = ok ? ((uint32_t)(oc * 8) * cstride + (uint32_t)(h * a.W + w) * 4u) : 0x7fffffffu;
#pragma unroll
            for (int j = 0; j < 8; ++j) xr[r][j] = __builtin_amdgcn_raw_buffer_load_b32(rs, vo, j * cstride, 0);
        }
    };
    auto load_w = [&](int kb, int chunk) __attribute__((always_inline)) {
        const uint4* wc = wpk + ((int64_t)kb * a.nchunks + chunk) * kfr;
        if constexpr (MC) {
#define PO2Q_W_LOAD(r, reg)                  \
    {                                        \
        const int e = tid + (r) * kThreads;  \
        reg = wc[e < kfr ? e : kfr - 1];     \
    }
            PO2Q_W_ALL(PO2Q_W_LOAD)
#undef PO2Q_W_LOAD
        } else {  // one (k-block, chunk) for the whole launch: straight to LDS, once
            uint4* wl0 = reinterpret_cast<uint4*>(lds + a.w_off);
            for (int e = tid; e < kfr; e += kThreads) wl0[e] = wc[e];
        }
    };

    floatx4 acc[NJ][NT];
#pragma unroll
    for (int g = 0; g < NJ; ++g)
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[g][t] = floatx4{0.f, 0.f, 0.f, 0.f};

    const float scale = *scale_p;
    uint4* wl = reinterpret_cast<uint4*>(lds + a.w_off);
    const int trash = zero_off + 16;  // per-plane 16-byte slot for padding items

    // Epilogue of a finished tile: D[row = pixel 4*(lane>>4)+i][col = channel lane&15]
    auto epilogue = [&](const TileCoord& tcs) __attribute__((always_inline)) {
        const int64_t PQ = (int64_t)a.P * a.Q;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
            const int k = tcs.kb * 16 * NT + nt * 16 + (lane & 15);
            const bool kv = k < a.K;
            const float bk = bias_l[tcs.kb * 16 * NT + nt * 16 + (lane & 15)];
            float* yk = y + ((int64_t)tcs.n * a.K + k) * PQ;
#pragma unroll
            for (int g = 0; g < NJ; ++g) {
                if (a.vec) {
                    const int pp = tcs.p0 + (ep[g] >> 16), qq = tcs.q0 + (ep[g] & 0xffff);
                    if (kv && ep[g] >= 0 && pp < a.P && qq < a.Q) {
                        floatx4 r4;
                        r4[0] = acc[g][nt][0] * scale + bk;
                        r4[1] = acc[g][nt][1] * scale + bk;
                        r4[2] = acc[g][nt][2] * scale + bk;
                        r4[3] = acc[g][nt][3] * scale + bk;
                        store_f4(yk + (int64_t)pp * a.Q + qq, r4);
                    }
                } else {
                    const int i0 = (wave * NJ + g) * 16 + 4 * o;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int idx = i0 + i;
                        const int pl = idx / a.TQ, ql = idx - (idx / a.TQ) * a.TQ;
                        const int pp = tcs.p0 + pl, qq = tcs.q0 + ql;
                        if (kv && idx < npix && pp < a.P && qq < a.Q)
                            store_f1(yk + (int64_t)pp * a.Q + qq, acc[g][nt][i] * scale + bk);
                    }
                }
                acc[g][nt] = floatx4{0.f, 0.f, 0.f, 0.f};
            }
        }
    };

    // Work items (tile v, chunk); past the end the "next" item repeats the last one
    // (its prefetch is a harmless re-load), so no control-flow join follows a load.
    struct Item {
        int v, chunk;
        bool valid;
        TileCoord tc;
    };
    auto next_item = [&](const Item& it) __attribute__((always_inline)) {
        Item n = it;
        n.chunk = it.chunk + 1;
        if (n.chunk == a.nchunks) {
            n.chunk = 0;
            n.v = it.v + (int)gridDim.x;
        }
        n.valid = it.valid && n.v < T;
        if (!n.valid) {
            n.v = it.v;
            n.chunk = it.chunk;
        } else if (n.v != it.v) {
            n.tc = tile_of(n.v, a);
        }
        return n;
    };

    Item cur{v, 0, true, tile_of(v, a)};
    Item n1 = next_item(cur);
    TileCoord done_tc = cur.tc;  // tile whose finished sums sit in acc (stored one step later)
    bool done = false;
    load_x(xa, cur.tc, 0);
    load_w(cur.tc.kb, 0);
    if constexpr (PD == 2) load_x(xb, n1.tc, n1.chunk);

    // One work item, in this order (vmcnt counts loads AND stores in issue order, so
    // the stores of the previous tile go out BEFORE the next prefetch: waiting for a
    // prefetch at the split then never waits for just-issued stores):
    //   barrier | x regs -> split -> LDS, weights -> LDS | barrier |
    //   stores of the previous tile | prefetch (PD items ahead) | MFMAs of this item
    // PD == 2 alternates two x register sets (xa: even items, xb: odd), so two items'
    // loads are in flight across each MFMA phase.
    auto step = [&](uint32_t (&xr)[kXI][8], const Item& it, const Item& pf) __attribute__((always_inline)) {
        __syncthreads();  // the previous item's MFMAs are done with LDS
#pragma unroll
        for (int r = 0; r < kXI; ++r) {  // unconditional: padding items go to the trash slot
            const uint32_t d = pk[r];
            const int hp = (int)((d >> 20) & 0x7ffu) * a.WW + (int)((d >> 8) & 0xfffu);
            uint4 hi, mid, lo;
            if (kDbg(a) & 2) {
                hi = make_uint4(xr[r][0], xr[r][1], xr[r][2], xr[r][3]);
                mid = lo = make_uint4(xr[r][4], xr[r][5], xr[r][6], xr[r][7]);
            } else {
                split3(xr[r], hi, mid, lo);
            }
            const int ad = (d >> 31) ? x_addr<CC>(hp, (int)(d & 0xffu)) : trash;
            *reinterpret_cast<uint4*>(lds + ad) = hi;
            *reinterpret_cast<uint4*>(lds + a.plane + ad) = mid;
            *reinterpret_cast<uint4*>(lds + 2 * a.plane + ad) = lo;
        }
        if constexpr (MC) {
#define PO2Q_W_STORE(r, reg)                 \
    {                                        \
        const int e = tid + (r) * kThreads;  \
        wl[e < kfr ? e : kfr - 1] = reg;     \
    }
            PO2Q_W_ALL(PO2Q_W_STORE)
#undef PO2Q_W_STORE
        }
        __syncthreads();

        if (done && !(kDbg(a) & 8)) {
            epilogue(done_tc);
            done = false;
            // drain this wave's stores before the next prefetch goes out: measured
            // faster than letting the loads queue behind them (HBM read/write turnaround)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }

        // ---- prefetch: x of item `pf` into the registers just split, weights of the next item
        load_x(xr, pf.tc, pf.chunk);
        if constexpr (MC) {
            const Item nw = PD == 2 ? n1 : pf;
            load_w(nw.tc.kb, nw.chunk);
        }

        // ---- MFMAs over this chunk: k = (tap, channel), 32 per step
        auto kstep = [&](int ks, int toff, int coct, bool pad) __attribute__((always_inline)) {
            bf16x8 bw[NT];
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
                bw[nt] = __builtin_bit_cast(bf16x8, wl[(ks * NT + nt) * 64 + lane]);
#pragma unroll
            for (int g = 0; g < NJ; ++g) {
                const int ad = pad ? zero_off : x_addr<CC>(hp0[g] + toff, coct);
                const bf16x8 a0 = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(lds + ad));
                const bf16x8 a1 = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(lds + a.plane + ad));
                const bf16x8 a2 =
                    __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(lds + 2 * a.plane + ad));
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) {
                    acc[g][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bw[nt], acc[g][nt], 0, 0, 0);
                    acc[g][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bw[nt], acc[g][nt], 0, 0, 0);
                    acc[g][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2, bw[nt], acc[g][nt], 0, 0, 0);
                }
            }
        };
        if (kDbg(a) & 1) {
        } else if constexpr (KS > 0) {
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) kstep(ks, tpx[ks], tco[ks], (padm >> ks) & 1u);
        } else {
            for (int ks = 0; ks < ksteps; ++ks) {
                const int oi = ks * 4 + o;
                const int t = oi / OCT;
                const bool pad = t >= a.taps;
                kstep(ks, pad ? 0 : tapt[t], oi % OCT, pad);
            }
        }
        if (it.chunk == a.nchunks - 1) {
            done = true;
            done_tc = it.tc;
        }
    };

    if constexpr (PD == 1) {
        while (true) {
            step(xa, cur, n1);
            if (!n1.valid) break;
            cur = n1;
            n1 = next_item(n1);
        }
    } else {
        while (true) {
            Item n2 = next_item(n1);
            step(xa, cur, n2);
            if (!n1.valid) break;
            cur = n1;
            n1 = n2;
            n2 = next_item(n1);
            step(xb, cur, n2);
            if (!n1.valid) break;
            cur = n1;
            n1 = n2;
        }
    }
    if (!(kDbg(a) & 8)) epilogue(done_tc);
#undef PO2Q_W_ALL
}

// ------------------------------------------------------------------ planning --
static int cdiv(int a, int b) { return (a + b - 1) / b; }

static size_t x3_lds(const ConvPlan& p, int NT, int HH, int WW) {
    const int plane = HH * WW * p.SB + 32;
    return (size_t)3 * plane + (size_t)p.steps * NT * 1024 + 64 * sizeof(int) +
           (size_t)p.kblocks * 16 * NT * sizeof(float);
}

void x3_candidates(const ConvPlan& base, int mode, int bits, int fsr, std::vector<PlanCand>& out) {
    if (mode == 0 || base.groups != 1) return;
    if (bits < 1 || bits > 16) return;
    const long lo = (long)fsr - (1L << (bits - 1)), hi = (long)fsr - 1;
    if (lo < -126 || hi > 127) return;  // +-2^e must be a normal bf16
    ConvPlan p = base;
    p.taps = p.R * p.S;
    if (p.taps > 64) return;
    if ((int64_t)p.H * p.W * 4 * 32 >= (1LL << 31)) return;  // 32-bit buffer offsets per chunk
    p.CC = (p.taps == 1 && p.C > 16) ? 32 : 16;
    const int OCT = p.CC / 8;
    p.steps = cdiv(p.taps * OCT, 4);
    p.SB = 2 * p.CC;
    p.NT = p.K <= 16 ? 1 : (p.K <= 32 ? 2 : 4);
    while (p.NT > 1 && p.steps * p.NT * 64 > kWI * kThreads) p.NT >>= 1;
    if (p.steps * p.NT * 64 > kWI * kThreads) return;
    p.kblocks = cdiv(p.K, 16 * p.NT);
    p.nchunks = cdiv(p.C, p.CC);
    p.kind = KIND_BF16X3;
    p.vrx = 0; p.PS = 0; p.MI = 0;
    p.dma_d0 = p.dma_nck = p.dma_ni = p.dma_nw = p.dma_waves = p.dma_ov = 0;

    // tile candidates (override: PO2Q_X3_TILE="NJ,TP,TQ", a tuning knob; it must pass
    // the same validity checks as every searched candidate)
    const char* env = getenv("PO2Q_X3_TILE");
    int fnj = 0, ftp = 0, ftq = 0;
    bool forced = env && sscanf(env, "%d,%d,%d", &fnj, &ftp, &ftq) == 3;
    auto consider = [&](int nj, int tp, int tq, int pd) {
        if (nj == 7 && p.NT > 1) return;  // > 256 VGPRs: spills
        if (pd == 2 && nj > 4) return;    // two x register sets: NJ <= 4
        if (tp < 1 || tq < 1 || tp * tq != 64 * nj) return;
        if (forced && (nj != fnj || tp != ftp || tq != ftq)) return;
        const int px = 64 * nj;
        const int HH = (tp - 1) * p.sh + (p.R - 1) * p.dh + 1;
        const int WW = (tq - 1) * p.sw + (p.S - 1) * p.dw + 1;
        const size_t lds = x3_lds(p, p.NT, HH, WW);
        if (lds > 64 * 1024) return;
        if (HH * WW * (p.CC / 8) > kXI * kThreads) return;  // staged items per thread
        if (HH >= 2048 || WW >= 4096) return;               // packed staging descriptors
        const int tP = cdiv(p.P, tp), tQ = cdiv(p.Q, tq);
        const double launched = (double)tP * tQ * px;
        const double waste = launched / ((double)p.P * p.Q);
        const double halo = (double)tP * tQ * HH * WW / ((double)p.P * p.Q * p.sh * p.sw);
        const int bpc = std::min<int>(8, (int)((160 * 1024) / lds));
        const int waves = std::min(bpc * 4, 32);
        double cost = waste + 0.35 * (halo - 1.0);
        if (waves < 8) cost += 0.15 * (8 - waves) / 4.0;
        if (tq % 16 && tq != p.Q) cost += 0.05;
        if (tq % 4) cost += 0.1;
        cost += 0.02 * (8.0 / nj);  // per-tile fixed costs (barriers, descriptors)
        if (pd == 2) cost -= 0.01;  // deeper prefetch: same tile, more loads in flight
        const double blocks = (double)p.N * p.kblocks * tP * tQ;
        if (blocks < 1024) cost += 0.5 * (1024 - blocks) / 1024;
        if (blocks > INT_MAX) return;
        ConvPlan c = p;
        c.NJ = nj; c.TP = tp; c.TQ = tq;
        c.pd = pd;
        c.tilesP = tP; c.tilesQ = tQ;
        c.HH = HH; c.WW = WW; c.WWp = WW;
        c.plane = HH * WW * p.SB + 32;  // + zero slot + trash slot
        c.lds_bytes = lds;
        // packed bf16 fragments: [kb][chunk][ks][nt][lane][8] -> 4-byte words
        c.packed_floats = (int64_t)p.kblocks * p.nchunks * p.steps * p.NT * 64 * 4;
        c.blocks = (int64_t)blocks;
        out.push_back({cost, c});
    };
    const int njs[] = {1, 2, 4, 7};
    for (int pass = 0; pass < 2 && out.empty(); ++pass, forced = false)  // an invalid override is ignored
        for (int nj : njs)
            for (int tq = 1; tq <= std::min(p.Q, 64 * nj); ++tq)
                if ((64 * nj) % tq == 0)
                    for (int pd : {1, 2}) consider(nj, 64 * nj / tq, tq, pd);
    std::stable_sort(out.begin(), out.end(), [](const PlanCand& a, const PlanCand& b) { return a.cost < b.cost; });
}

bool plan_bf16x3(ConvPlan& p, int mode, int bits, int fsr) {
    std::vector<PlanCand> c;
    x3_candidates(p, mode, bits, fsr, c);
    if (c.empty()) return false;
    p = c[0].plan;
    return true;
}

template <int CC, int NT, int NJ, int KS, bool MC, int PD>
static hipError_t launch_x3p(const ConvPlan& p, const X3Args& a, const float* x, const uint16_t* packed,
                             const float* scale, const float* bias, float* y, hipStream_t s) {
    // persistent grid: as many blocks as can be co-resident (LDS / VGPR occupancy)
    int per_cu = 0, dev = 0, cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, conv_bf16x3<CC, NT, NJ, KS, MC, PD>, kThreads,
                                                     p.lds_bytes) !=
            hipSuccess || per_cu < 1)
        per_cu = 1;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
        cus = 256;
    const int64_t grid = std::min<int64_t>(p.blocks, (int64_t)per_cu * cus);
    hipLaunchKernelGGL((conv_bf16x3<CC, NT, NJ, KS, MC, PD>), dim3((unsigned)grid), dim3(kThreads), p.lds_bytes, s,
                       x, reinterpret_cast<const uint4*>(packed), scale, bias, y, a);
    return hipGetLastError();
}

template <int CC, int NT, int NJ, int KS, bool MC>
static hipError_t launch_x3(const ConvPlan& p, const X3Args& a, const float* x, const uint16_t* packed,
                            const float* scale, const float* bias, float* y, hipStream_t s) {
    if constexpr (NJ <= 4)
        if (p.pd == 2) return launch_x3p<CC, NT, NJ, KS, MC, 2>(p, a, x, packed, scale, bias, y, s);
    return launch_x3p<CC, NT, NJ, KS, MC, 1>(p, a, x, packed, scale, bias, y, s);
}

template <int CC, int NT, int NJ>
static hipError_t launch_x3_ks(const ConvPlan& p, const X3Args& a, const float* x, const uint16_t* packed,
                               const float* scale, const float* bias, float* y, hipStream_t s) {
    const bool mc = p.nchunks > 1 || p.kblocks > 1;
    if (p.steps == 1)
        return mc ? launch_x3<CC, NT, NJ, 1, true>(p, a, x, packed, scale, bias, y, s)
                  : launch_x3<CC, NT, NJ, 1, false>(p, a, x, packed, scale, bias, y, s);
    if constexpr (CC == 16)
        if (p.steps == 5)
            return mc ? launch_x3<CC, NT, NJ, 5, true>(p, a, x, packed, scale, bias, y, s)
                      : launch_x3<CC, NT, NJ, 5, false>(p, a, x, packed, scale, bias, y, s);
    return mc ? launch_x3<CC, NT, NJ, 0, true>(p, a, x, packed, scale, bias, y, s)
              : launch_x3<CC, NT, NJ, 0, false>(p, a, x, packed, scale, bias, y, s);
}

template <int CC, int NT>
static hipError_t launch_x3_nj(const ConvPlan& p, const X3Args& a, const float* x, const uint16_t* packed,
                               const float* scale, const float* bias, float* y, hipStream_t s) {
    switch (p.NJ) {
        case 1: return launch_x3_ks<CC, NT, 1>(p, a, x, packed, scale, bias, y, s);
        case 2: return launch_x3_ks<CC, NT, 2>(p, a, x, packed, scale, bias, y, s);
        case 4: return launch_x3_ks<CC, NT, 4>(p, a, x, packed, scale, bias, y, s);
        default:
            if constexpr (NT == 1) return launch_x3_ks<CC, NT, 7>(p, a, x, packed, scale, bias, y, s);
            return hipErrorInvalidValue;  // the planner never pairs NJ = 7 with NT > 1 (register file)
    }
}

template <int CC>
static hipError_t launch_x3_nt(const ConvPlan& p, const X3Args& a, const float* x, const uint16_t* packed,
                               const float* scale, const float* bias, float* y, hipStream_t s) {
    switch (p.NT) {
        case 1: return launch_x3_nj<CC, 1>(p, a, x, packed, scale, bias, y, s);
        case 2: return launch_x3_nj<CC, 2>(p, a, x, packed, scale, bias, y, s);
        default: return launch_x3_nj<CC, 4>(p, a, x, packed, scale, bias, y, s);
    }
}

hipError_t launch_conv_bf16x3(const ConvPlan& p, const float* x, const uint16_t* packed, const float* scale,
                              const float* bias, float* y, hipStream_t s) {
    X3Args a;
    a.N = p.N; a.C = p.C; a.H = p.H; a.W = p.W; a.K = p.K; a.P = p.P; a.Q = p.Q;
    a.sh = p.sh; a.sw = p.sw; a.ph = p.ph; a.pw = p.pw; a.dh = p.dh; a.dw = p.dw; a.R = p.R; a.S = p.S;
    a.TP = p.TP; a.TQ = p.TQ; a.tilesP = p.tilesP; a.tilesQ = p.tilesQ; a.kblocks = p.kblocks;
    a.nchunks = p.nchunks; a.HH = p.HH; a.WW = p.WW; a.ksteps = p.steps; a.taps = p.taps;
    a.plane = p.plane;
    a.w_off = 3 * p.plane;
    a.tap_off = a.w_off + p.steps * p.NT * 1024;
    a.bias_off = a.tap_off + 64 * (int)sizeof(int);
    a.vec = (p.Q % 4 == 0 && p.TQ % 4 == 0) ? 1 : 0;
    a.nblocks = (int)p.blocks;
    a.remap = (p.blocks % 8 == 0) ? 1 : 0;
    const char* dbg = getenv("PO2Q_X3_DEBUG");  // timing diagnostics only: outputs are wrong
    a.dbg = dbg ? atoi(dbg) : 0;
    if (p.CC == 16) return launch_x3_nt<16>(p, a, x, packed, scale, bias, y, s);
    return launch_x3_nt<32>(p, a, x, packed, scale, bias, y, s);
}

}  // namespace po2q
