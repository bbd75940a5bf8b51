// bf16x3 conv, LDS-DMA pipelined (the production path for ResNet-shaped layers).
//
// Same arithmetic as po2q_conv_x3.hip (exact +-2^e bf16 weights x exact 3-way bf16
// activation split, fp32 accumulation on v_mfma_f32_16x16x32_bf16; reference:
// QuantizedConv2d.forward, models/quantized_conv.py:32-38), different data movement:
//
//   * x is fetched by LDS-DMA (`buffer_load_dwordx4 ... lds`) straight into a raw
//     fp32 ring in LDS, TWO work items ahead -- no VGPRs hold in-flight data, so a
//     512-thread block keeps ~2 tiles of HBM reads in flight while it computes.
//     Out-of-image pixels and channels >= C read 0 through the buffer descriptor's
//     range check (the conv's zero padding), so the DMA issue is branch-free.
//   * a split pass turns the raw tile into the three bf16 planes
//     [halo pixel][16 ch] (hi / mid / lo) the MFMA fragments are read from;
//   * the MFMA schedule is either the row-reuse one (3x3 / stride 1 / <= 16 output
//     channels: the 5 A fragments of a halo row feed up to 3 output rows, weights
//     stay in registers) or the generic k-step one (any R x S, 16*NT channels);
//   * every global memory instruction inside the loop is inline asm (DMA loads,
//     epilogue stores), so hipcc inserts no vmcnt waits of its own: the only waits
//     are the counted `s_waitcnt vmcnt(N)` below, one per work item, which retire
//     exactly the DMA of the item about to be split (N = the vm ops issued after it:
//     the next item's DMA and the stores in between; every lane stores on every
//     epilogue slot -- lanes without an output hit a dummy workspace word -- so the
//     per-wave store count is exact).
//
// Work items: (output tile, 16-channel chunk), persistent grid (one 512-thread
// block per CU), block b walks tiles b, b + grid, ... (XCD-aware tile order).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "po2q_internal.h"
#include "po2q_x3_dev.h"

namespace po2q {

constexpr int kPMaxNI = 8;      // max x-DMA instructions per wave per item
constexpr int kPMaxNW = 8;      // max weight-DMA instructions per wave per item (multi-chunk)
constexpr int kPXS = 3;         // max split items per thread per work item

struct X3PArgs {
    int N, C, H, W, K, P, Q, sh, sw, ph, pw, dh, dw, R, S;
    int TP, TQ, tilesP, tilesQ, kblocks, nchunks, HH, WW, ksteps, taps;
    int plane;               // bytes per bf16 plane (halo pixels * 32 + zero slot + trash slot)
    int nck, d0;             // 16-byte chunks per raw halo row; w0 - (aligned window start), floats
    int ni, nw;              // x / weight DMA instructions per wave per work item
    int raw_off, raw_slot;   // LDS byte offset of the raw ring (2 slots) / bytes per slot
    int w_off, w_slot;       // LDS byte offset of the weight ring (3 slots if multi-chunk) / bytes per slot
    int bias_off, tap_off;
    int vec, remap, nblocks;
    uint32_t m_tiles[2], m_tq[2], m_kb[2];  // udiv_magic multipliers (lo, hi) for tiles, tilesQ, kblocks
    int dbg;  // timing diagnostics only (PO2Q_X3_DEBUG): 1 no MFMA, 2 no split, 4 no DMA, 8 no stores
    unsigned* stamps;  // PO2Q_STAMPS diagnostic builds only: per-wave phase cycle sums
};

// Diagnostic build (-DPO2Q_STAMPS, `make stamps`): s_memtime phase stamps, one
// statement each (guide §7 "In-kernel stamps"); never in the product build.
#ifdef PO2Q_STAMPS
#define PO2Q_STAMP(i)                                                                      \
    do {                                                                                   \
        __builtin_amdgcn_sched_barrier(0);                                                 \
        unsigned long long t_;                                                             \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");          \
        __builtin_amdgcn_sched_barrier(0);                                                 \
        ph_[i] += (unsigned)(t_ - tprev_);                                                 \
        tprev_ = t_;                                                                       \
    } while (0)
#else
#define PO2Q_STAMP(i) \
    do {              \
    } while (0)
#endif

// s_waitcnt vmcnt(n) for a wave-uniform runtime n (the instruction takes an
// immediate).  n > 63 waits for vmcnt(63): stricter, so still correct.
#define PO2Q_VM(n) \
    case n: asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory"); break;
__device__ __forceinline__ void wait_vmcnt(int n) {
    switch (n) {
        PO2Q_VM(0) PO2Q_VM(1) PO2Q_VM(2) PO2Q_VM(3) PO2Q_VM(4) PO2Q_VM(5) PO2Q_VM(6) PO2Q_VM(7)
        PO2Q_VM(8) PO2Q_VM(9) PO2Q_VM(10) PO2Q_VM(11) PO2Q_VM(12) PO2Q_VM(13) PO2Q_VM(14) PO2Q_VM(15)
        PO2Q_VM(16) PO2Q_VM(17) PO2Q_VM(18) PO2Q_VM(19) PO2Q_VM(20) PO2Q_VM(21) PO2Q_VM(22) PO2Q_VM(23)
        PO2Q_VM(24) PO2Q_VM(25) PO2Q_VM(26) PO2Q_VM(27) PO2Q_VM(28) PO2Q_VM(29) PO2Q_VM(30) PO2Q_VM(31)
        PO2Q_VM(32) PO2Q_VM(33) PO2Q_VM(34) PO2Q_VM(35) PO2Q_VM(36) PO2Q_VM(37) PO2Q_VM(38) PO2Q_VM(39)
        PO2Q_VM(40) PO2Q_VM(41) PO2Q_VM(42) PO2Q_VM(43) PO2Q_VM(44) PO2Q_VM(45) PO2Q_VM(46) PO2Q_VM(47)
        PO2Q_VM(48) PO2Q_VM(49) PO2Q_VM(50) PO2Q_VM(51) PO2Q_VM(52) PO2Q_VM(53) PO2Q_VM(54) PO2Q_VM(55)
        PO2Q_VM(56) PO2Q_VM(57) PO2Q_VM(58) PO2Q_VM(59) PO2Q_VM(60) PO2Q_VM(61) PO2Q_VM(62)
        default: asm volatile("s_waitcnt vmcnt(63)" ::: "memory"); break;
    }
}
#undef PO2Q_VM

// One LDS-DMA wave instruction: 64 lanes x 16 bytes from rsrc + voff -> LDS [m0 + 16*lane].
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t lds_addr) {
    asm volatile("s_nop 4\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %2, 0 offen lds"
                 ::"v"(voff), "s"(lds_addr), "s"(rs)
                 : "memory");
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* base, int64_t bytes) {
    const uintptr_t bp = reinterpret_cast<uintptr_t>(base);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)bp);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(bp >> 32));
    const int nrec = __builtin_amdgcn_readfirstlane((int)(bytes > 0x7fffffffLL ? 0x7fffffffLL : (bytes < 0 ? 0 : bytes)));
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uintptr_t)hi << 32) | lo), (short)0, nrec,
                                             0x00020000);
}

// (image, k-block, tile origin) of virtual tile v (XCD-aware order, as tile_of).
__device__ __forceinline__ TileCoord tile_of_p(int v, const X3PArgs& a) {
    if (a.remap) v = (v & 7) * (a.nblocks >> 3) + (v >> 3);
    const int tiles = a.tilesP * a.tilesQ;
    const int nk = (int)udiv_magic((uint32_t)v, a.m_tiles[0], a.m_tiles[1]);
    const int tile = v - nk * tiles;
    const int tp = (int)udiv_magic((uint32_t)tile, a.m_tq[0], a.m_tq[1]);
    TileCoord t;
    t.n = (int)udiv_magic((uint32_t)nk, a.m_kb[0], a.m_kb[1]);
    t.kb = nk - t.n * a.kblocks;
    t.p0 = tp * a.TP;
    t.q0 = (tile - tp * a.tilesQ) * a.TQ;
    return t;
}

template <int WV, int NT, int NJ, int VRX, int KS, bool MC, bool OV>
__global__ __launch_bounds__(WV * 64, 1) void conv_x3p(const float* __restrict__ x, const uint4* __restrict__ wpk,
                                                         const float* __restrict__ scale_p,
                                                         const float* __restrict__ bias, float* __restrict__ y,
                                                         X3PArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    constexpr int CC = 16;
    constexpr int OCT = 2;
    constexpr bool VR = VRX > 0;
    constexpr int KSR = KS ? KS : 1;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int o = lane >> 4;
    const int T = a.nblocks;
    int v0 = blockIdx.x;
    if (v0 >= T) return;
    const int npix = a.TP * a.TQ;
    const int hw_halo = a.HH * a.WW;
    const int zero_off = hw_halo * 32;
    const int trash = zero_off + 16;
    const int items = hw_halo * OCT;
    const int ksteps = KS ? KS : a.ksteps;
    const int kfr = ksteps * NT * 64;  // weight fragments (uint4) per (k-block, chunk)
    const int64_t HWi = (int64_t)a.H * a.W;
    const uint32_t hw4 = (uint32_t)HWi * 4u;
    const uint32_t lds_base = (uint32_t)(uintptr_t)lds;

    // ---- one-time LDS init: zero slots, tap table, bias
    if (tid < (OV ? 6 : 3)) *reinterpret_cast<uint4*>(lds + tid * a.plane + zero_off) = make_uint4(0u, 0u, 0u, 0u);
    int* tapt = reinterpret_cast<int*>(lds + a.tap_off);
    if (!VR && !KS && tid < a.taps) {
        const int r = tid / a.S, s = tid - (tid / a.S) * a.S;
        tapt[tid] = r * a.dh * a.WW + s * a.dw;
    }
    float* bias_l = reinterpret_cast<float*>(lds + a.bias_off);
    for (int k = tid; k < a.kblocks * 16 * NT; k += (WV * 64)) bias_l[k] = (bias && k < a.K) ? bias[k] : 0.0f;

    // ---- per-lane MFMA geometry
    int hp0[VR ? 1 : NJ], ep[NJ];
    if constexpr (VR) {  // wave (wx, wy): columns wx*16 .. +15, rows wy*NJ .. +NJ-1
        const int wx = wave % VRX, wy = wave / VRX;
        hp0[0] = (wy * NJ) * a.WW + wx * 16 + (lane & 15);
#pragma unroll
        for (int g = 0; g < NJ; ++g) ep[g] = ((wy * NJ + g) << 16) | (wx * 16 + 4 * o);
    } else {  // wave owns tile-linear pixel groups wave*NJ .. +NJ-1 (16 pixels each)
#pragma unroll
        for (int g = 0; g < NJ; ++g) {
            int slot = (wave * NJ + g) * 16 + (lane & 15);
            if (slot >= npix) slot = 0;
            const int pl = slot / a.TQ, ql = slot - (slot / a.TQ) * a.TQ;
            hp0[g] = pl * a.sh * a.WW + ql * a.sw;
            const int i0 = (wave * NJ + g) * 16 + 4 * o;
            ep[g] = (i0 < npix) ? (((i0 / a.TQ) << 16) | (i0 - (i0 / a.TQ) * a.TQ)) : -1;
        }
    }
    int tpx[KSR], tco[KSR];
    unsigned padm = 0;
    if constexpr (!VR && KS > 0) {
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

    // ---- split-pass descriptors: item it = (channel octet, halo pixel); raw byte
    // offset of its first channel (8 channels at stride HH * nck * 16) and plane address
    const int raw_cstride = a.HH * a.nck * 16;
    int sraw[kPXS], spl[kPXS];
#pragma unroll
    for (int r = 0; r < kPXS; ++r) {
        const int it = tid + r * (WV * 64);
        const int oc = it / hw_halo, hp = it - (it / hw_halo) * hw_halo;
        const int hh = hp / a.WW, ww = hp - (hp / a.WW) * a.WW;
        const bool ok = it < items;
        sraw[r] = ok ? (8 * oc * raw_cstride + hh * a.nck * 16 + (a.d0 + ww) * 4) : 0;
        spl[r] = ok ? x_addr<CC>(hp, oc) : trash;
    }
    // ---- x DMA descriptors: instruction ii = wave + 8r covers raw chunks ii*64 + lane,
    // chunk = (channel c, halo row hh, 16-byte column k); packed (valid, c, hh, k)
    const int chunks = CC * a.HH * a.nck;
    uint32_t dpk[kPMaxNI];
#pragma unroll
    for (int r = 0; r < kPMaxNI; ++r) {
        const int q = (wave + WV * r) * 64 + lane;
        const int c = q / (a.HH * a.nck), rem = q - (q / (a.HH * a.nck)) * (a.HH * a.nck);
        const int hh = rem / a.nck, k = rem - (rem / a.nck) * a.nck;
        dpk[r] = (q < chunks) ? (0x80000000u | ((uint32_t)c << 24) | ((uint32_t)hh << 12) | (uint32_t)k) : 0u;
    }

    // Work items (tile, chunk); past the end: marked invalid, re-issue the last valid
    // item's DMA (never consumed) so every wave issues the same DMA count per item.
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
            n.tc = tile_of_p(n.v, a);
        }
        return n;
    };

    // x: raw fp32 halo tile of item `it` -> raw slot `slot` (a.ni DMA instructions per wave)
    auto issue_x = [&](const Item& it, int slot) __attribute__((always_inline)) {
        const int h0 = it.tc.p0 * a.sh - a.ph;
        const int ws = it.tc.q0 * a.sw - a.pw - a.d0;  // 16-byte aligned window start (floats)
        const float* base = x + ((int64_t)it.tc.n * a.C + it.chunk * CC) * HWi;
        const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(base, (int64_t)(a.C - it.chunk * CC) * HWi * 4);
        const uint32_t dst = lds_base + a.raw_off + slot * a.raw_slot + wave * 1024;
#pragma unroll
        for (int r = 0; r < kPMaxNI; ++r) {
            if (r < a.ni) {  // wave-uniform
                const uint32_t d = dpk[r];
                const int c = (int)((d >> 24) & 0x3fu), hh = (int)((d >> 12) & 0xfffu), k = (int)(d & 0xfffu);
                const int h = h0 + hh, w = ws + 4 * k;
                const bool ok = (d >> 31) && ((unsigned)h < (unsigned)a.H) && ((unsigned)w < (unsigned)a.W);
                // 32-bit: the planner bounds 16 channels of one image below 2^31 bytes
                const uint32_t vo = ok ? ((uint32_t)c * hw4 + (uint32_t)(h * a.W + w) * 4u) : 0x80000000u;
                dma16(rs, vo, dst + r * WV * 1024);
            }
        }
    };
    // weights of (k-block, chunk) -> weight slot (multi-chunk only; a.nw DMAs per wave)
    auto issue_w = [&](const Item& it, int slot) __attribute__((always_inline)) {
        const uint4* src = wpk + ((int64_t)it.tc.kb * a.nchunks + it.chunk) * kfr;
        const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(src, (int64_t)kfr * 16);
        const uint32_t dst = lds_base + a.w_off + slot * a.w_slot + wave * 1024;
#pragma unroll
        for (int r = 0; r < kPMaxNW; ++r) {
            if (r < a.nw) {
                const uint32_t e = (uint32_t)((wave + WV * r) * 64 + lane);
                dma16(rs, e * 16u, dst + r * WV * 1024);
            }
        }
    };

    floatx4 acc[NJ][NT];
#pragma unroll
    for (int g = 0; g < NJ; ++g)
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[g][t] = floatx4{0.f, 0.f, 0.f, 0.f};
    const float scale = *scale_p;

    Item i0{v0, 0, true, tile_of_p(v0, a)};
    Item i1 = next_item(i0);
    int wslot = 0;  // weight slot of i0 (multi-chunk ring of 3)
    if constexpr (!MC) {  // one k-block for the whole launch: every chunk's weights -> LDS once
        uint4* wl0 = reinterpret_cast<uint4*>(lds + a.w_off);
        const uint4* src = wpk + ((int64_t)i0.tc.kb * a.nchunks) * kfr;
        for (int e = tid; e < kfr * a.nchunks; e += (WV * 64)) wl0[e] = src[e];
    }
    __syncthreads();  // LDS init + weights visible; plain loads all retired (vmcnt(0))
    bf16x8 bvr[VR ? 15 : 1];
    if constexpr (VR && !MC) {
#pragma unroll
        for (int f = 0; f < 15; ++f)
            bvr[f] = __builtin_bit_cast(bf16x8, reinterpret_cast<const uint4*>(lds + a.w_off)[f * 64 + lane]);
    }
    // split of one thread's r-th item: raw fp32 (8 channels) -> bf16 hi / mid / lo planes
    auto split_one = [&](int r, const unsigned char* raw, unsigned char* pl) __attribute__((always_inline)) {
        if (r * (WV * 64) < items) {  // block-uniform
            uint32_t b[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) b[j] = *reinterpret_cast<const uint32_t*>(raw + sraw[r] + j * raw_cstride);
            uint4 hi, mid, lo;
            split3(b, hi, mid, lo);
            *reinterpret_cast<uint4*>(pl + spl[r]) = hi;
            *reinterpret_cast<uint4*>(pl + a.plane + spl[r]) = mid;
            *reinterpret_cast<uint4*>(pl + 2 * a.plane + spl[r]) = lo;
        }
    };
    const int per_item = a.ni + (MC ? a.nw : 0);
    const int pset = 3 * a.plane;  // bytes per plane set (OV: two sets)
    int rslot = 0;   // raw slot of i0
    int younger;     // vm ops issued after the DMA the loop top waits for
    int pcur = 0;    // OV: plane set holding i0
    Item i2;         // OV: the item after i1 (its x DMA is in flight)
    if constexpr (OV) {
        // Overlapped pipeline: raw ring of 3, plane sets of 2.  Iteration j (item i0)
        // waits for x(i1) and w(i0), then issues x(i0 + 3) and w(i0 + 2) and runs the
        // MFMAs of i0 interleaved with the split of i1 -- one barrier per item.
        issue_x(i0, 0);
        if constexpr (MC) issue_w(i0, 0);
        issue_x(i1, 1);
        wait_vmcnt(a.ni + (MC ? a.nw : 0));  // x(i0) landed
        __builtin_amdgcn_s_barrier();
#pragma unroll
        for (int r = 0; r < kPXS; ++r) split_one(r, lds + a.raw_off, lds);
        i2 = next_item(i1);
        if constexpr (MC) issue_w(i1, 1);
        issue_x(i2, 2);
        younger = a.ni + (MC ? a.nw : 0);
    } else {
        issue_x(i0, 0);
        if constexpr (MC) issue_w(i0, 0);
        issue_x(i1, 1);
        if constexpr (MC) issue_w(i1, 1);
        younger = per_item;  // next item's DMA (+ stores)
    }

    TileCoord done_tc = i0.tc;
    bool done = false;
    const int st_per_tile = NJ * NT * (a.vec ? 1 : 4);

    // Every lane stores on every (nt, g): lanes without an output write to a dummy
    // workspace slot, so each wave issues exactly NJ * NT (vec) or 4 * NJ * NT stores
    // per tile and the counted vmcnt waits below know how many stores are in flight.
    float* dummy = reinterpret_cast<float*>(reinterpret_cast<uintptr_t>(scale_p) + 64);
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
                    const bool ok = kv && ep[g] >= 0 && pp < a.P && qq < a.Q;
                    floatx4 r4;
                    r4[0] = acc[g][nt][0] * scale + bk;
                    r4[1] = acc[g][nt][1] * scale + bk;
                    r4[2] = acc[g][nt][2] * scale + bk;
                    r4[3] = acc[g][nt][3] * scale + bk;
                    store_f4(ok ? yk + (int64_t)pp * a.Q + qq : dummy, r4);
                } else {
                    const int i0p = (ep[g] >> 16) * a.TQ + (ep[g] & 0xffff);
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int idx = i0p + i;
                        const int pl = idx / a.TQ, ql = idx - (idx / a.TQ) * a.TQ;
                        const int pp = tcs.p0 + pl, qq = tcs.q0 + ql;
                        const bool ok = kv && ep[g] >= 0 && idx < npix && pp < a.P && qq < a.Q;
                        store_f1(ok ? yk + (int64_t)pp * a.Q + qq : dummy, acc[g][nt][i] * scale + bk);
                    }
                }
                acc[g][nt] = floatx4{0.f, 0.f, 0.f, 0.f};
            }
        }
    };

#ifdef PO2Q_STAMPS
    unsigned ph_[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long tprev_;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(tprev_)::"memory");
#endif
    while (true) {
        // (1) this item's DMA has landed (the next item's DMA may stay in flight), and
        //     every wave is past the previous item's MFMAs
        PO2Q_STAMP(0);
        if constexpr (OV) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's split writes
        wait_vmcnt(younger);
        PO2Q_STAMP(1);
        __builtin_amdgcn_s_barrier();
        PO2Q_STAMP(2);
        // (2) split: raw fp32 -> bf16 hi / mid / lo planes (OV: interleaved with the MFMAs below)
        if constexpr (!OV) {
            if (!(kDbg(a) & 2)) {
                const unsigned char* raw = lds + a.raw_off + rslot * a.raw_slot;
#pragma unroll
                for (int r = 0; r < kPXS; ++r) split_one(r, raw, lds);
            }
            PO2Q_STAMP(3);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();  // planes complete, raw slot free
            PO2Q_STAMP(4);
        }
        const unsigned char* pl = lds + pcur * pset;  // planes of i0
        const int rnext = (rslot == 2) ? 0 : rslot + 1;
        const unsigned char* raw_n = lds + a.raw_off + rnext * a.raw_slot;  // OV: raw of i1
        unsigned char* pl_n = lds + (pcur ^ 1) * pset;                      // OV: planes for i1
        const bool do_split = OV && !(kDbg(a) & 2);
        const unsigned char* wcur = lds + a.w_off + (MC ? wslot * a.w_slot : i0.chunk * kfr * 16);
        if constexpr (VR) {
            if (MC || a.nchunks > 1) {
#pragma unroll
                for (int f = 0; f < 15; ++f)
                    bvr[f] = __builtin_bit_cast(bf16x8, reinterpret_cast<const uint4*>(wcur)[f * 64 + lane]);
            }
        }
        // (3) stores of the previous tile (older than the next DMA in vmcnt order)
        const int nst = (done && !(kDbg(a) & 8)) ? st_per_tile : 0;
        if (done && !(kDbg(a) & 8)) {
            epilogue(done_tc);
            done = false;
        }
        PO2Q_STAMP(5);
        younger = nst + per_item;  // after the next item's DMA: these stores + the DMA below
        // (4) DMA of the item after next into the raw slot just split (+ its weights);
        //     OV: x of the item three ahead, weights of the item two ahead
        Item i3;
        if constexpr (OV) {
            i3 = next_item(i2);
        } else {
            i2 = next_item(i1);
        }
        if (!(kDbg(a) & 4)) {
            if constexpr (OV) {
                issue_x(i3, rslot);
            } else {
                issue_x(i2, rslot);
            }
            if constexpr (MC) issue_w(i2, wslot == 0 ? 2 : wslot - 1);  // (wslot + 2) % 3
        } else {
            younger = nst;
        }
        PO2Q_STAMP(6);
        // (5) MFMAs of this item
        if (kDbg(a) & 1) {
        } else if constexpr (VR) {
            const int rowb = a.WW * 32;
            const int oct16 = ((lane >> 4) & 1) * 16;
            const bool upper = lane >= 32;
            const int hm = hp0[0] * 32 + oct16 + (upper ? a.plane : 0);
            const int l01 = (hp0[0] + (upper ? 1 : 0)) * 32 + oct16 + 2 * a.plane;
            const int l2 = upper ? zero_off : (hp0[0] + 2) * 32 + oct16 + 2 * a.plane;
            const int l2s = upper ? 0 : rowb;
            auto ld = [&](int ad) __attribute__((always_inline)) {
                return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(pl + ad));
            };
            bf16x8 cur[5], nxt[5];
            cur[0] = ld(hm); cur[1] = ld(hm + 32); cur[2] = ld(hm + 64); cur[3] = ld(l01); cur[4] = ld(l2);
#pragma unroll
            for (int ir = 0; ir < NJ + 2; ++ir) {
                if (ir + 1 < NJ + 2) {
                    const int ro = (ir + 1) * rowb;
                    nxt[0] = ld(hm + ro); nxt[1] = ld(hm + ro + 32); nxt[2] = ld(hm + ro + 64);
                    nxt[3] = ld(l01 + ro); nxt[4] = ld(l2 + (ir + 1) * l2s);
                }
#pragma unroll
                for (int r = 0; r < 3; ++r) {
                    const int i = ir - r;
                    if (i >= 0 && i < NJ) {
#pragma unroll
                        for (int f = 0; f < 5; ++f)
                            acc[i][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur[f], bvr[r * 5 + f], acc[i][0], 0, 0, 0);
                    }
                }
                if (ir < kPXS && do_split) split_one(ir, raw_n, pl_n);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int f = 0; f < 5; ++f) cur[f] = nxt[f];
            }
        } else {
            const uint4* wl = reinterpret_cast<const uint4*>(wcur);
            auto kstep = [&](int ks, int toff, int coct, bool pad) __attribute__((always_inline)) {
                bf16x8 bw[NT];
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) bw[nt] = __builtin_bit_cast(bf16x8, wl[(ks * NT + nt) * 64 + lane]);
#pragma unroll
                for (int g = 0; g < NJ; ++g) {
                    const int ad = pad ? zero_off : x_addr<CC>(hp0[g] + toff, coct);
                    const bf16x8 a0 = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(pl + ad));
                    const bf16x8 a1 = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(pl + a.plane + ad));
                    const bf16x8 a2 =
                        __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(pl + 2 * a.plane + ad));
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt) {
                        acc[g][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bw[nt], acc[g][nt], 0, 0, 0);
                        acc[g][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bw[nt], acc[g][nt], 0, 0, 0);
                        acc[g][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2, bw[nt], acc[g][nt], 0, 0, 0);
                    }
                }
            };
            if constexpr (KS > 0) {
#pragma unroll
                for (int ks = 0; ks < KS; ++ks) {
                    kstep(ks, tpx[ks], tco[ks], (padm >> ks) & 1u);
                    if (ks < kPXS && do_split) split_one(ks, raw_n, pl_n);
                }
                if (KS < kPXS && do_split)
#pragma unroll
                    for (int r = KS; r < kPXS; ++r) split_one(r, raw_n, pl_n);
            } else {
                if (do_split)
#pragma unroll
                    for (int r = 0; r < kPXS; ++r) split_one(r, raw_n, pl_n);
                for (int ks = 0; ks < ksteps; ++ks) {
                    const int oi = ks * 4 + o;
                    const int t = oi / OCT;
                    const bool pad = t >= a.taps;
                    kstep(ks, pad ? 0 : tapt[t], oi % OCT, pad);
                }
            }
        }
        PO2Q_STAMP(7);
        if (i0.chunk == a.nchunks - 1) {
            done = true;
            done_tc = i0.tc;
        }
#ifdef PO2Q_STAMPS
        ph_[8] += 1;
#endif
        if (!i1.valid) break;
        i0 = i1;
        i1 = i2;
        if constexpr (OV) {
            i2 = i3;
            rslot = rnext;
            pcur ^= 1;
        } else {
            rslot ^= 1;
        }
        if constexpr (MC) wslot = (wslot == 2) ? 0 : wslot + 1;
    }
    if (!(kDbg(a) & 8)) epilogue(done_tc);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the trailing (unconsumed) DMAs
#ifdef PO2Q_STAMPS
    if (lane == 0 && a.stamps)
        for (int i = 0; i < 9; ++i) a.stamps[((size_t)blockIdx.x * WV + wave) * 9 + i] = ph_[i];
#endif
}

// ------------------------------------------------------------------ planning --
static int cdivp(int a, int b) { return (a + b - 1) / b; }

// Eligible: po2/po2+ (bf16x3 already planned), groups == 1, taps <= 64, W % 4 == 0,
// a 16-byte-aligned input window per tile (TQ * stride % 4 == 0), K block bias in LDS.
void x3p_candidates(const ConvPlan& base, std::vector<PlanCand>& out) {
    const char* wenv = getenv("PO2Q_X3P_WAVES");  // tuning knob: 4 or 8 waves per block
    const ConvPlan& p = base;
    if (p.groups != 1 || p.taps > 64 || p.W % 4 || p.K > 1024) return;
    if ((int64_t)p.H * p.W * 4 * 16 >= (1LL << 31)) return;
    const bool vr_ok = p.R == 3 && p.S == 3 && p.sh == 1 && p.sw == 1 && p.dh == 1 && p.dw == 1 && p.K <= 16;
    const int cc = 16;
    const int nchunks = cdivp(p.C, cc);
    const int ksteps_k = cdivp(p.taps * 2, 4);
    int NT = p.K <= 16 ? 1 : (p.K <= 32 ? 2 : 4);
    while (NT > 1 && ksteps_k * NT * 64 > kPMaxNW * 4 * 64) NT >>= 1;
    const int kblocks = cdivp(p.K, 16 * NT);
    const bool multi = nchunks > 1 || kblocks > 1;
    const int d0 = ((p.pw % 4) + 4) % 4 == 0 ? 0 : 4 - (p.pw % 4);  // w0 - aligned window start

    const char* env = getenv("PO2Q_X3P_TILE");  // "NJ,TP,TQ,VRX" tuning knob
    int fnj = 0, ftp = 0, ftq = 0, fvr = -1;
    if (env && sscanf(env, "%d,%d,%d,%d", &fnj, &ftp, &ftq, &fvr) != 4) fvr = -1;
    // mc: weights streamed per (k-block, chunk) item through a ring of 3 LDS slots;
    // otherwise (one k-block) every chunk's weights stay resident in LDS for the launch
    auto consider = [&](int waves, int nj, int tp, int tq, int vrx, bool ov, bool mc) {
        if (mc != multi && !(multi && kblocks == 1)) return;
        if (vrx && (!vr_ok || NT != 1)) return;
        if (tp * tq != 16 * waves * nj) return;
        if ((tq * p.sw) % 4) return;
        if (vrx && (vrx > waves || tq != 16 * vrx || tp != nj * (waves / vrx))) return;
        if (wenv && atoi(wenv) != waves) return;
        if (fvr >= 0 && !(nj == fnj && tp == ftp && tq == ftq && vrx == fvr)) return;
        const int HH = (tp - 1) * p.sh + (p.R - 1) * p.dh + 1;
        const int WW = (tq - 1) * p.sw + (p.S - 1) * p.dw + 1;
        if (HH >= 4096 || WW >= 4096) return;
        const int nck = cdivp(d0 + WW, 4);
        const int ni = cdivp(cc * HH * nck, 64 * waves);
        if (ni > kPMaxNI) return;
        if (cdivp(HH * WW * 2, 64 * waves) > kPXS) return;
        const int plane = HH * WW * 32 + 32;
        const int raw_slot = ni * waves * 1024;
        const int steps = vrx ? 15 : ksteps_k;
        const int wfr = steps * NT * 64;
        const int nw = cdivp(wfr, 64 * waves);
        if (mc && nw > kPMaxNW) return;
        const int w_slot = (mc ? nw * waves * 1024 : wfr * 16 * nchunks);
        const size_t lds = (size_t)(ov ? 6 : 3) * plane + (ov ? 3 : 2) * (size_t)raw_slot +
                           (mc ? 3 : 1) * (size_t)w_slot + 4096 + 256;
        if (lds > 160 * 1024) return;
        const int bpc = (int)((160 * 1024) / lds);  // co-resident blocks per CU (LDS)
        const int tP = cdivp(p.P, tp), tQ = cdivp(p.Q, tq);
        const double waste = (double)tP * tQ * tp * tq / ((double)p.P * p.Q);
        const double halo = (double)tP * tQ * HH * WW / ((double)p.P * p.Q * p.sh * p.sw);
        double cost = waste + 0.35 * (halo - 1.0) + (vrx ? -0.2 : 0.0) + (ov ? -0.1 : 0.0) + (mc ? 0.2 : 0.0);
        if (bpc < 2) cost += 0.3;  // one block per CU: its barriers stall every wave in the same phase
        const double blocks = (double)p.N * kblocks * tP * tQ;
        if (blocks < 512) cost += 0.5 * (512 - blocks) / 512;
        if (blocks >= (1 << 20) || (double)tP * tQ >= (1 << 20)) return;  // udiv_magic range
        ConvPlan c = p;
        c.kind = KIND_BF16X3_DMA;
        c.CC = cc; c.SB = 32; c.NT = NT; c.kblocks = kblocks; c.nchunks = nchunks;
        c.NJ = nj; c.TP = tp; c.TQ = tq; c.vrx = vrx;
        c.steps = steps;
        c.tilesP = tP; c.tilesQ = tQ;
        c.HH = HH; c.WW = WW; c.WWp = WW; c.PS = 0; c.MI = 0;
        c.plane = plane;
        c.dma_d0 = d0; c.dma_nck = nck; c.dma_waves = waves; c.dma_ni = ni;
        c.dma_nw = mc ? nw : 0;
        c.dma_ov = ov ? 1 : 0;
        c.lds_bytes = lds;
        c.packed_floats = (int64_t)kblocks * nchunks * steps * NT * 64 * 4;
        c.blocks = (int64_t)blocks;
        out.push_back({cost, c});
    };
    for (int waves : {4, 8})
        for (int nj : {1, 2, 4}) {
            const int px = 16 * waves * nj;
            for (bool ov : {false, true})
                for (bool mc : {false, true}) {
                    for (int tq = 4; tq <= std::min(p.Q + 3, px); tq += 4)
                        if (px % tq == 0) consider(waves, nj, px / tq, tq, 0, ov, mc);
                    for (int vrx : {1, 2, 4, 8})
                        if (vrx <= waves) consider(waves, nj, nj * (waves / vrx), 16 * vrx, vrx, ov, mc);
                }
        }
    std::stable_sort(out.begin(), out.end(), [](const PlanCand& a, const PlanCand& b) { return a.cost < b.cost; });
}

bool plan_bf16x3_dma(ConvPlan& p) {
    std::vector<PlanCand> c;
    x3p_candidates(p, c);
    if (c.empty()) return false;
    p = c[0].plan;
    return true;
}

template <int WV, int NT, int NJ, int VRX, int KS, bool MC, bool OV>
static hipError_t launch_p1(const ConvPlan& p, const X3PArgs& a, const float* x, const uint16_t* packed,
                            const float* scale, const float* bias, float* y, hipStream_t s) {
    auto kern = conv_x3p<WV, NT, NJ, VRX, KS, MC, OV>;
    if (p.lds_bytes > 64 * 1024) {
        const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)p.lds_bytes);
        if (e != hipSuccess) return e;
    }
    int dev = 0, cus = 256, per_cu = 1;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
        cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, WV * 64, p.lds_bytes) != hipSuccess ||
        per_cu < 1)
        per_cu = 1;
    const int64_t grid = std::min<int64_t>(p.blocks, (int64_t)per_cu * cus);
#ifdef PO2Q_STAMPS
    X3PArgs as = a;
    const size_t nst = (size_t)grid * WV * 9;
    if (getenv("PO2Q_STAMPS") && hipMalloc(&as.stamps, nst * 4) == hipSuccess) {
        (void)hipMemsetAsync(as.stamps, 0, nst * 4, s);
        hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(WV * 64), p.lds_bytes, s, x,
                           reinterpret_cast<const uint4*>(packed), scale, bias, y, as);
        std::vector<unsigned> h(nst);
        (void)hipStreamSynchronize(s);
        (void)hipMemcpy(h.data(), as.stamps, nst * 4, hipMemcpyDeviceToHost);
        (void)hipFree(as.stamps);
        double sum[9] = {0};
        for (size_t i = 0; i < nst; ++i) sum[i % 9] += h[i];
        const double waves = (double)grid * WV, items = sum[8] / waves;
        static const char* names[8] = {"loop-top", "vmcnt-wait", "barrier1", "split", "barrier2",
                                       "epilogue", "dma-issue", "mfma"};
        double tot = 0;
        for (int i = 0; i < 8; ++i) tot += sum[i];
        fprintf(stderr, "[po2q stamps] grid=%lld waves/block=%d items/wave=%.1f cycles/item/wave=%.0f\n",
                (long long)grid, WV, items, tot / waves / items);
        for (int i = 0; i < 8; ++i)
            fprintf(stderr, "  %-11s %8.0f cyc/item  %5.1f%%\n", names[i], sum[i] / waves / items,
                    100.0 * sum[i] / tot);
        return hipGetLastError();
    }
#endif
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(WV * 64), p.lds_bytes, s, x,
                       reinterpret_cast<const uint4*>(packed), scale, bias, y, a);
    return hipGetLastError();
}

template <int WV, int NT, int NJ, int VRX, int KS, bool MC>
static hipError_t launch_p(const ConvPlan& p, const X3PArgs& a, const float* x, const uint16_t* packed,
                           const float* scale, const float* bias, float* y, hipStream_t s) {
    return p.dma_ov ? launch_p1<WV, NT, NJ, VRX, KS, MC, true>(p, a, x, packed, scale, bias, y, s)
                    : launch_p1<WV, NT, NJ, VRX, KS, MC, false>(p, a, x, packed, scale, bias, y, s);
}

template <int WV, int NT, int NJ>
static hipError_t launch_p_k(const ConvPlan& p, const X3PArgs& a, const float* x, const uint16_t* packed,
                             const float* scale, const float* bias, float* y, hipStream_t s) {
    const bool mc = p.dma_nw > 0;  // weights streamed per item (else resident)
    if (p.steps == 5)
        return mc ? launch_p<WV, NT, NJ, 0, 5, true>(p, a, x, packed, scale, bias, y, s)
                  : launch_p<WV, NT, NJ, 0, 5, false>(p, a, x, packed, scale, bias, y, s);
    return mc ? launch_p<WV, NT, NJ, 0, 0, true>(p, a, x, packed, scale, bias, y, s)
              : launch_p<WV, NT, NJ, 0, 0, false>(p, a, x, packed, scale, bias, y, s);
}

template <int WV>
static hipError_t launch_p_w(const ConvPlan& p, const X3PArgs& a, const float* x, const uint16_t* packed,
                             const float* scale, const float* bias, float* y, hipStream_t s) {
    if (p.vrx) {
        const bool mcv = p.dma_nw > 0;
#define PO2Q_PVR(NJ_, VRX_)                                                                         \
    if constexpr (VRX_ <= WV)                                                                       \
        if (p.NJ == NJ_ && p.vrx == VRX_)                                                           \
            return mcv ? launch_p<WV, 1, NJ_, VRX_, 0, true>(p, a, x, packed, scale, bias, y, s)    \
                       : launch_p<WV, 1, NJ_, VRX_, 0, false>(p, a, x, packed, scale, bias, y, s);
        PO2Q_PVR(1, 1) PO2Q_PVR(1, 2) PO2Q_PVR(1, 4) PO2Q_PVR(1, 8)
        PO2Q_PVR(2, 1) PO2Q_PVR(2, 2) PO2Q_PVR(2, 4) PO2Q_PVR(2, 8)
        PO2Q_PVR(4, 1) PO2Q_PVR(4, 2) PO2Q_PVR(4, 4) PO2Q_PVR(4, 8)
#undef PO2Q_PVR
        return hipErrorInvalidValue;
    }
    switch (p.NT * 8 + p.NJ) {
        case 9: return launch_p_k<WV, 1, 1>(p, a, x, packed, scale, bias, y, s);
        case 10: return launch_p_k<WV, 1, 2>(p, a, x, packed, scale, bias, y, s);
        case 12: return launch_p_k<WV, 1, 4>(p, a, x, packed, scale, bias, y, s);
        case 17: return launch_p_k<WV, 2, 1>(p, a, x, packed, scale, bias, y, s);
        case 18: return launch_p_k<WV, 2, 2>(p, a, x, packed, scale, bias, y, s);
        case 20: return launch_p_k<WV, 2, 4>(p, a, x, packed, scale, bias, y, s);
        case 33: return launch_p_k<WV, 4, 1>(p, a, x, packed, scale, bias, y, s);
        case 34: return launch_p_k<WV, 4, 2>(p, a, x, packed, scale, bias, y, s);
        case 36: return launch_p_k<WV, 4, 4>(p, a, x, packed, scale, bias, y, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_conv_bf16x3_dma(const ConvPlan& p, const float* x, const uint16_t* packed, const float* scale,
                                  const float* bias, float* y, hipStream_t s) {
    X3PArgs a;
    a.N = p.N; a.C = p.C; a.H = p.H; a.W = p.W; a.K = p.K; a.P = p.P; a.Q = p.Q;
    a.sh = p.sh; a.sw = p.sw; a.ph = p.ph; a.pw = p.pw; a.dh = p.dh; a.dw = p.dw; a.R = p.R; a.S = p.S;
    a.TP = p.TP; a.TQ = p.TQ; a.tilesP = p.tilesP; a.tilesQ = p.tilesQ; a.kblocks = p.kblocks;
    a.nchunks = p.nchunks; a.HH = p.HH; a.WW = p.WW; a.ksteps = p.steps; a.taps = p.taps;
    a.plane = p.plane;
    a.nck = p.dma_nck; a.d0 = p.dma_d0; a.ni = p.dma_ni; a.nw = p.dma_nw;
    const bool mc = p.dma_nw > 0;
    const int wfr = p.steps * p.NT * 64;
    a.raw_off = (p.dma_ov ? 6 : 3) * p.plane;
    a.raw_slot = p.dma_ni * p.dma_waves * 1024;
    a.w_off = a.raw_off + (p.dma_ov ? 3 : 2) * a.raw_slot;
    a.w_slot = mc ? p.dma_nw * p.dma_waves * 1024 : wfr * 16 * p.nchunks;
    a.bias_off = a.w_off + (mc ? 3 : 1) * a.w_slot;
    a.tap_off = a.bias_off + 4096;
    a.vec = (p.Q % 4 == 0 && p.TQ % 4 == 0) ? 1 : 0;
    a.nblocks = (int)p.blocks;
    a.remap = (p.blocks % 8 == 0) ? 1 : 0;
    auto magic = [](uint32_t (&m)[2], int d) {
        const uint64_t v = (1ULL << 40) / (uint64_t)d + 1;
        m[0] = (uint32_t)v;
        m[1] = (uint32_t)(v >> 32);
    };
    magic(a.m_tiles, p.tilesP * p.tilesQ);
    magic(a.m_tq, p.tilesQ);
    magic(a.m_kb, p.kblocks);
    const char* dbg = getenv("PO2Q_X3_DEBUG");  // timing diagnostics only: outputs are wrong
    a.dbg = dbg ? atoi(dbg) : 0;
    a.stamps = nullptr;
    return p.dma_waves == 4 ? launch_p_w<4>(p, a, x, packed, scale, bias, y, s)
                            : launch_p_w<8>(p, a, x, packed, scale, bias, y, s);
}

}  // namespace po2q
