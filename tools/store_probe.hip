// Store-pattern probe (tuning aid, not part of the product): writes an NCHW fp32
// tensor [N][C][H][W] the way a row-marching conv block does -- block = (image,
// strip of SW columns, segment of RB rows), per row every channel's SW-column
// piece -- and times nothing itself (tools/store_probe.py times the launches).
//   mode 0: per row, wave w stores channels [w*C/4, (w+1)*C/4): one instruction =
//           CPI channels x SW*4 bytes (CPI = 256 / SW)
//   mode 1: contiguous: each block writes RB*SW*C... consecutive floats (copy-like)
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

__device__ __forceinline__ __amdgpu_buffer_rsrc_t mk(void* p, uint32_t bytes) {
    const uintptr_t bp = reinterpret_cast<uintptr_t>(p);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)bp);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(bp >> 32));
    void* b = reinterpret_cast<void*>(((uintptr_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(b, (short)0, bytes, 0x00020000);
}

typedef float f4 __attribute__((ext_vector_type(4)));

template <int NT>
__device__ __forceinline__ void st(__amdgpu_buffer_rsrc_t rs, uint32_t vo, f4 v) {
    if constexpr (NT)
        asm volatile("buffer_store_dwordx4 %0, %1, %2, 0 offen nt" ::"v"(v), "v"(vo), "s"(rs));
    else
        asm volatile("buffer_store_dwordx4 %0, %1, %2, 0 offen" ::"v"(v), "v"(vo), "s"(rs));
}

template <int NT>
__global__ __launch_bounds__(256) void probe_rows(float* y, int N, int C, int H, int W, int SW, int RB, int bar) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nstrip = (W + SW - 1) / SW, nseg = (H + RB - 1) / RB;
    int blk = blockIdx.x;
    blk = (blk & 7) * (int)(gridDim.x >> 3) + (blk >> 3);
    if (blk >= N * nseg * nstrip) return;
    const int strip = blk % nstrip, seg = (blk / nstrip) % nseg, n = blk / (nstrip * nseg);
    const uint32_t plane = (uint32_t)H * W;
    const __amdgpu_buffer_rsrc_t rs = mk(y + (int64_t)n * C * plane, C * plane * 4u);
    const int lpc = SW / 4;            // lanes per channel
    const int cpi = 64 / lpc;          // channels per instruction
    const int cpw = C / 4;             // channels per wave
    const int q = strip * SW + 4 * (lane % lpc);
    const f4 v = f4{1.f, 2.f, 3.f, 4.f};
    for (int r = seg * RB; r < min(H, seg * RB + RB); ++r) {
        for (int i = 0; i < cpw / cpi; ++i) {
            const int c = wave * cpw + i * cpi + lane / lpc;
            const uint32_t vo = (q < W) ? ((uint32_t)c * plane + (uint32_t)r * W + q) * 4u : 0x7fffffffu;
            st<NT>(rs, vo, v);
        }
        if (bar) __builtin_amdgcn_s_barrier();
    }
}

// mode 2: the same walk, loading the input row's pieces (to VGPRs) before storing
template <int NT>
__global__ __launch_bounds__(256) void probe_rows_ld(const float* x, float* y, int N, int C, int H, int W, int SW,
                                                     int RB, int bar) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nstrip = (W + SW - 1) / SW, nseg = (H + RB - 1) / RB;
    int blk = blockIdx.x;
    blk = (blk & 7) * (int)(gridDim.x >> 3) + (blk >> 3);
    if (blk >= N * nseg * nstrip) return;
    const int strip = blk % nstrip, seg = (blk / nstrip) % nseg, n = blk / (nstrip * nseg);
    const uint32_t plane = (uint32_t)H * W;
    const __amdgpu_buffer_rsrc_t rs = mk(y + (int64_t)n * C * plane, C * plane * 4u);
    const __amdgpu_buffer_rsrc_t rx = mk(const_cast<float*>(x) + (int64_t)n * C * plane, C * plane * 4u);
    const int lpc = SW / 4, cpi = 64 / lpc, cpw = C / 4;
    const int q = strip * SW + 4 * (lane % lpc);
    f4 acc = f4{0.f, 0.f, 0.f, 0.f};
    for (int r = seg * RB; r < min(H, seg * RB + RB); ++r) {
        for (int i = 0; i < cpw / cpi; ++i) {
            const int c = wave * cpw + i * cpi + lane / lpc;
            const uint32_t vo = (q < W) ? ((uint32_t)c * plane + (uint32_t)r * W + q) * 4u : 0x7fffffffu;
            if constexpr (NT == 2) {  // LDS-DMA into a per-wave 1 KiB slot
                extern __shared__ unsigned char lds_[];
                const uint32_t m0 = (uint32_t)(uintptr_t)lds_ + (uint32_t)(wave * 1024 * 4 + i * 1024);
                asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %2, 0 offen lds"
                             ::"v"(vo), "s"(m0), "s"(rx) : "memory");
            } else {
                f4 v;
                asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(v) : "v"(vo), "s"(rx) : "memory");
                acc += v;
            }
        }
        for (int i = 0; i < cpw / cpi; ++i) {
            const int c = wave * cpw + i * cpi + lane / lpc;
            const uint32_t vo = (q < W) ? ((uint32_t)c * plane + (uint32_t)r * W + q) * 4u : 0x7fffffffu;
            asm volatile("s_waitcnt vmcnt(0)" : "+v"(acc));
            st<0>(rs, vo, acc);
        }
        if (bar) __builtin_amdgcn_s_barrier();
    }
}

__global__ __launch_bounds__(256) void probe_contig(float* y, int64_t n4) {
    f4* p = reinterpret_cast<f4*>(y);
    for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) p[i] = f4{1.f, 2.f, 3.f, 4.f};
}

}  // namespace

extern "C" int probe_launch(float* y, const float* x, int mode, int N, int C, int H, int W, int SW, int RB, int bar,
                            int nt) {
    if (mode == 1) {
        hipLaunchKernelGGL(probe_contig, dim3(256 * 16), dim3(256), 0, 0, y, (int64_t)N * C * H * W / 4);
        return (int)hipGetLastError();
    }
    const int nstrip = (W + SW - 1) / SW, nseg = (H + RB - 1) / RB;
    const int items = N * nseg * nstrip;
    const int blocks = (items + 7) / 8 * 8;
    if (mode == 2) {
        if (nt == 2)
            hipLaunchKernelGGL(probe_rows_ld<2>, dim3(blocks), dim3(256), 16384, 0, x, y, N, C, H, W, SW, RB, bar);
        else
            hipLaunchKernelGGL(probe_rows_ld<0>, dim3(blocks), dim3(256), 0, 0, x, y, N, C, H, W, SW, RB, bar);
        return (int)hipGetLastError();
    }
    if (nt)
        hipLaunchKernelGGL(probe_rows<1>, dim3(blocks), dim3(256), 0, 0, y, N, C, H, W, SW, RB, bar);
    else
        hipLaunchKernelGGL(probe_rows<0>, dim3(blocks), dim3(256), 0, 0, y, N, C, H, W, SW, RB, bar);
    return (int)hipGetLastError();
}
