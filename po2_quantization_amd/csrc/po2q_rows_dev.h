// Device helpers shared by the row-streaming bf16x3 conv kernels
// (po2q_conv_rows.hip, po2q_conv_rowsk.hip).  Not part of the C ABI.
//
// Every global access inside their row loops is inline asm (no compiler-visible load or
// store there), so hipcc's vmcnt bookkeeping -- which at a loop header falls back to
// vmcnt(0), i.e. waits for every store and every prefetch, and which would place a
// vmcnt(0) before the first use of any builtin load issued behind asm DMAs -- stays out of
// the picture: each step waits with one exact, hand-counted `s_waitcnt vmcnt`.  Residual
// rows go through LDS by the same counted DMAs (po2q_conv_rowsf.hip, po2q_conv_rowsk.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "po2q_x3_dev.h"

namespace po2q {

// One LDS-DMA wave instruction: lane l's 16 (or 4) bytes at rsrc + voff land at LDS
// m0 + 16*l (4*l).  `s_waitcnt lgkmcnt(0)` first: earlier reads of the slot being
// refilled have returned.  NT: non-temporal (streaming) load policy -- on this
// layer's once-read activations an nt copy moves the same bytes ~10 % faster
// (tools/copy_probe.hip, profiles/r02_copy_probe.jsonl).
template <bool NT = false>
__device__ __forceinline__ void rows_dma16(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t soff,
                                           uint32_t lds_addr) {
    if constexpr (NT)
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_nop 4\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
                     "buffer_load_dwordx4 %0, %2, %3 offen nt lds"
                     ::"v"(voff), "s"(lds_addr), "s"(rs), "s"(soff)
                     : "memory");
    else
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_nop 4\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
                     "buffer_load_dwordx4 %0, %2, %3 offen lds"
                     ::"v"(voff), "s"(lds_addr), "s"(rs), "s"(soff)
                     : "memory");
}
template <bool NT = false>
__device__ __forceinline__ void rows_dma4(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t lds_addr) {
    if constexpr (NT)
        asm volatile("s_nop 4\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dword %0, %2, 0 offen nt lds"
                     ::"v"(voff), "s"(lds_addr), "s"(rs)
                     : "memory");
    else
        asm volatile("s_nop 4\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dword %0, %2, 0 offen lds"
                     ::"v"(voff), "s"(lds_addr), "s"(rs)
                     : "memory");
}
// out-of-range voffset (>= the descriptor's size): the store is dropped, yet counted
template <bool NTS = false>
__device__ __forceinline__ void rows_store(__amdgpu_buffer_rsrc_t rs, uint32_t vo, floatx4 v) {
    if constexpr (NTS)
        asm volatile("buffer_store_dwordx4 %0, %1, %2, 0 offen nt\n\ts_nop 1" ::"v"(v), "v"(vo), "s"(rs));
    else
        asm volatile("buffer_store_dwordx4 %0, %1, %2, 0 offen\n\ts_nop 1" ::"v"(v), "v"(vo), "s"(rs));
}
template <int N>
__device__ __forceinline__ void rows_wait() {
    static_assert(N >= 0 && N <= 63, "vm ops issued after a row's DMAs");
#define PO2Q_RW(n) \
    if constexpr (N == n) asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory");
    PO2Q_RW(0) PO2Q_RW(1) PO2Q_RW(2) PO2Q_RW(3) PO2Q_RW(4) PO2Q_RW(5) PO2Q_RW(6) PO2Q_RW(7)
    PO2Q_RW(8) PO2Q_RW(9) PO2Q_RW(10) PO2Q_RW(11) PO2Q_RW(12) PO2Q_RW(13) PO2Q_RW(14) PO2Q_RW(15)
    PO2Q_RW(16) PO2Q_RW(17) PO2Q_RW(18) PO2Q_RW(19) PO2Q_RW(20) PO2Q_RW(21) PO2Q_RW(22) PO2Q_RW(23)
    PO2Q_RW(24) PO2Q_RW(25) PO2Q_RW(26) PO2Q_RW(27) PO2Q_RW(28) PO2Q_RW(29) PO2Q_RW(30) PO2Q_RW(31)
    PO2Q_RW(32) PO2Q_RW(33) PO2Q_RW(34) PO2Q_RW(35) PO2Q_RW(36) PO2Q_RW(37) PO2Q_RW(38) PO2Q_RW(39)
    PO2Q_RW(40) PO2Q_RW(41) PO2Q_RW(42) PO2Q_RW(43) PO2Q_RW(44) PO2Q_RW(45) PO2Q_RW(46) PO2Q_RW(47)
    PO2Q_RW(48) PO2Q_RW(49) PO2Q_RW(50) PO2Q_RW(51) PO2Q_RW(52) PO2Q_RW(53) PO2Q_RW(54) PO2Q_RW(55)
    PO2Q_RW(56) PO2Q_RW(57) PO2Q_RW(58) PO2Q_RW(59) PO2Q_RW(60) PO2Q_RW(61) PO2Q_RW(62) PO2Q_RW(63)
#undef PO2Q_RW
}

// Wave-uniform buffer descriptor of `bytes` (< 2^31) starting at p.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rows_rsrc(const void* p, int bytes) {
    const uintptr_t bp = reinterpret_cast<uintptr_t>(p);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)bp);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(bp >> 32));
    void* b = reinterpret_cast<void*>(((uintptr_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(b, (short)0, bytes, 0x00020000);
}

// Exact 3-way split of one fp32 value (split3 of po2q_x3_dev.h, one lane value):
// the bf16 bit patterns of hi / mid / lo.
__device__ __forceinline__ void split1(uint32_t b, uint16_t& h, uint16_t& m, uint16_t& l) {
    const float xc = __builtin_amdgcn_fmed3f(__uint_as_float(b), -3.40282347e38f, 3.40282347e38f);
    const float r1 = xc - __uint_as_float(__float_as_uint(xc) & 0xffff0000u);
    const uint32_t mb = __float_as_uint(r1) & 0xffff0000u;
    const uint32_t lb = __float_as_uint(r1 - __uint_as_float(mb));
    h = (uint16_t)(b >> 16);
    m = (uint16_t)(mb >> 16);
    l = (uint16_t)(lb >> 16);
}

}  // namespace po2q
