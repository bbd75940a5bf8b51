// Device helpers shared by the bf16x3 conv kernels (po2q_conv_x3.hip,
// po2q_conv_x3p.hip): exact 3-way bf16 split, LDS plane addressing, asm
// epilogue stores, tile decoding.  Not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

// Timing-ablation switches (PO2Q_X3_DEBUG bits: 1 no MFMA, 2 no split, 4 no x loads,
// 8 no stores) exist only in the diagnostic build (-DPO2Q_DIAG=1, `make diag`): in the
// product build kDbg() is the constant 0, so none of the ablation branches -- which
// otherwise split the control flow the compiler's wait-count analysis sees -- is emitted.
#ifndef PO2Q_DIAG
#define PO2Q_DIAG 0
#endif

namespace po2q {

template <class Args>
__device__ __forceinline__ int kDbg(const Args& a) {
#if PO2Q_DIAG
    return a.dbg;
#else
    (void)a;
    return 0;
#endif
}

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

// Exact 3-way bf16 split of 8 fp32 values (bit patterns):
//   hi = x & 0xffff0000, r1 = x - hi (exact), mid = r1 & 0xffff0000, lo = r1 - mid.
// NaN needs no care (hi is NaN, and so is every product sum).
// +-inf would give r1 = inf - inf = NaN where the reference's product is +-inf, so
// r1 comes from the value clamped to +-FLT_MAX (v_med3: identity on every finite value):
// hi keeps +-inf, mid / lo are finite, and the products sum to +-inf as the reference's do.
// (a >> 16) | (b & 0xffff0000): the bf16 halves of a (low) and b (high) as one dword
__device__ __forceinline__ uint32_t pk_hi16(uint32_t a, uint32_t b) { return __builtin_amdgcn_perm(b, a, 0x07060302u); }

typedef float po2q_float2 __attribute__((ext_vector_type(2)));

// PK (default): the two subtractions of a value pair as one v_pk_add_f32 each; PK false: scalar
// v_sub_f32 per value (same IEEE results either way -- the conv pair keeps the scalar form, which
// measured faster there: its packed operands need register-pair moves)
template <bool PK = true>
__device__ __forceinline__ void split3(const uint32_t (&b)[8], uint4& hi, uint4& mid, uint4& lo) {
    uint32_t mb[8], lb[8];
    if constexpr (!PK) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float xc = __builtin_amdgcn_fmed3f(__uint_as_float(b[j]), -3.40282347e38f, 3.40282347e38f);
            const float r1 = xc - __uint_as_float(__float_as_uint(xc) & 0xffff0000u);
            mb[j] = __float_as_uint(r1) & 0xffff0000u;
            lb[j] = __float_as_uint(r1 - __uint_as_float(mb[j]));
        }
    } else {
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
        // +-inf: r1 from the value clamped to +-FLT_MAX (one v_med3 instead of a class test and
        // a select): finite mid / lo beside hi = +-inf, so every product sum stays +-inf.  The two
        // subtractions of a value pair are one packed v_pk_add_f32 each (same IEEE results).
        const float xc0 = __builtin_amdgcn_fmed3f(__uint_as_float(b[j]), -3.40282347e38f, 3.40282347e38f);
        const float xc1 = __builtin_amdgcn_fmed3f(__uint_as_float(b[j + 1]), -3.40282347e38f, 3.40282347e38f);
        const po2q_float2 xc = {xc0, xc1};
        const po2q_float2 h = {__uint_as_float(__float_as_uint(xc0) & 0xffff0000u),
                               __uint_as_float(__float_as_uint(xc1) & 0xffff0000u)};
        const po2q_float2 r1 = xc - h;
        mb[j] = __float_as_uint(r1.x) & 0xffff0000u;
        mb[j + 1] = __float_as_uint(r1.y) & 0xffff0000u;
        const po2q_float2 m = {__uint_as_float(mb[j]), __uint_as_float(mb[j + 1])};
        const po2q_float2 l = r1 - m;
        lb[j] = __float_as_uint(l.x);
        lb[j + 1] = __float_as_uint(l.y);
    }
    }
    // the upper halves of two dwords in one v_perm_b32 (the shift + and_or pair it replaces
    // cost two vector instructions per packed dword)
    hi = make_uint4(pk_hi16(b[0], b[1]), pk_hi16(b[2], b[3]), pk_hi16(b[4], b[5]), pk_hi16(b[6], b[7]));
    mid = make_uint4(pk_hi16(mb[0], mb[1]), pk_hi16(mb[2], mb[3]), pk_hi16(mb[4], mb[5]), pk_hi16(mb[6], mb[7]));
    lo = make_uint4(pk_hi16(lb[0], lb[1]), pk_hi16(lb[2], lb[3]), pk_hi16(lb[4], lb[5]), pk_hi16(lb[6], lb[7]));
}

// The same for 4 values (the epilogues' 4 channels of one pixel): 4 bf16 per plane, packed in
// channel order (low half = the even channel).
template <bool PK = true>
__device__ __forceinline__ void split4p(const uint32_t (&b)[4], uint2& hi, uint2& mid, uint2& lo) {
    uint32_t mb[4], lb[4];
    if constexpr (!PK) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float xc = __builtin_amdgcn_fmed3f(__uint_as_float(b[j]), -3.40282347e38f, 3.40282347e38f);
            const float r1 = xc - __uint_as_float(__float_as_uint(xc) & 0xffff0000u);
            mb[j] = __float_as_uint(r1) & 0xffff0000u;
            lb[j] = __float_as_uint(r1 - __uint_as_float(mb[j]));
        }
    } else {
#pragma unroll
    for (int j = 0; j < 4; j += 2) {
        const float xc0 = __builtin_amdgcn_fmed3f(__uint_as_float(b[j]), -3.40282347e38f, 3.40282347e38f);
        const float xc1 = __builtin_amdgcn_fmed3f(__uint_as_float(b[j + 1]), -3.40282347e38f, 3.40282347e38f);
        const po2q_float2 xc = {xc0, xc1};
        const po2q_float2 h = {__uint_as_float(__float_as_uint(xc0) & 0xffff0000u),
                               __uint_as_float(__float_as_uint(xc1) & 0xffff0000u)};
        const po2q_float2 r1 = xc - h;
        mb[j] = __float_as_uint(r1.x) & 0xffff0000u;
        mb[j + 1] = __float_as_uint(r1.y) & 0xffff0000u;
        const po2q_float2 m = {__uint_as_float(mb[j]), __uint_as_float(mb[j + 1])};
        const po2q_float2 l = r1 - m;
        lb[j] = __float_as_uint(l.x);
        lb[j + 1] = __float_as_uint(l.y);
    }
    }
    hi = make_uint2(pk_hi16(b[0], b[1]), pk_hi16(b[2], b[3]));
    mid = make_uint2(pk_hi16(mb[0], mb[1]), pk_hi16(mb[2], mb[3]));
    lo = make_uint2(pk_hi16(lb[0], lb[1]), pk_hi16(lb[2], lb[3]));
}

// Epilogue stores as inline asm: hipcc then leaves them out of its vmcnt
// bookkeeping.  Loads and stores share vmcnt on gfx950, and the stores of a tile
// are issued BEFORE the next prefetch, so every compiler wait for the prefetched
// x also covers these (older) stores; without this hipcc makes the following
// MFMAs wait for the stores' completion (register reuse WAR).  `s_nop 1` lets
// the store read its VGPRs before hipcc's next instruction may overwrite them.
__device__ __forceinline__ void store_f4(float* p, floatx4 v) {
    asm volatile("global_store_dwordx4 %0, %1, off\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void store_f1(float* p, float v) {
    asm volatile("global_store_dword %0, %1, off\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}

// LDS byte address of channel octet `coct` of halo pixel `hp` inside a plane.
template <int CC>
__device__ __forceinline__ int x_addr(int hp, int coct) {
    if constexpr (CC == 16) {
        return hp * 32 + coct * 16;
    } else {
        return hp * (2 * CC) + ((coct ^ ((hp >> 1) & 3)) << 4);
    }
}

// Output tile / image / k-block of virtual tile index v (XCD-aware when T % 8 == 0:
// the T/8 logical tiles an XCD owns are contiguous, so neighbouring tiles -- which
// share halo rows -- are processed under the same L2).
struct TileCoord {
    int n, kb, p0, q0;
};

template <class Args>
__device__ __forceinline__ TileCoord tile_of(int v, const Args& a) {
    if (a.remap) v = (v & 7) * (a.nblocks >> 3) + (v >> 3);
    const int tiles = a.tilesP * a.tilesQ;
    const int tile = v % tiles;
    v /= tiles;
    TileCoord t;
    t.kb = v % a.kblocks;
    t.n = v / a.kblocks;
    t.p0 = (tile / a.tilesQ) * a.TP;
    t.q0 = (tile % a.tilesQ) * a.TQ;
    return t;
}

// Division of a wave-uniform 0 <= x < 2^20 by 1 <= d < 2^20 through the host magic
// number m = floor(2^40 / d) + 1 (< 2^41, passed as lo / hi words): q = (x * m) >> 40,
// exact in that range (m*d - 2^40 <= d), three SALU ops instead of a ~30-instruction
// software division (the planner checks the ranges).
__device__ __forceinline__ uint32_t udiv_magic(uint32_t x, uint32_t mlo, uint32_t mhi) {
    return (__umulhi(x, mlo) + x * mhi) >> 8;
}

}  // namespace po2q
