// HBM copy-ceiling probe (tuning aid, not part of the product): how fast can ANY
// kernel move the stage-1 layer's bytes (256 x 16 x 224 x 224 fp32 = 822 MB read +
// 822 MB written) on this MI355X?  Standalone (no torch): hipcc -O3 --offload-arch=gfx950.
// Prints one JSON line per variant: median ms over reps and TB/s of read+written bytes.
//
//   gs<U,NTL,NTS>   grid-stride float4 copy, U loads in flight per lane before the stores
//   chunk<U,...>    block b copies its own contiguous chunk (CH float4), U loads in flight
//   rd / wr         read-only (sum, one conditional store) / write-only
//   planes<...>     the conv's geometry: wave = (image, segment of RB rows, 16 channel
//                   planes); per row it reads 16 x W floats (one 896-B run per channel)
//                   and writes the same amount 2 rows later (a 3x3 window's lag)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <functional>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

template <int NT>
__device__ __forceinline__ f4 ld(const f4* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    return *p;
}
template <int NT>
__device__ __forceinline__ void st(f4* p, f4 v) {
    if constexpr (NT)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}

template <int U, int NTL, int NTS>
__global__ __launch_bounds__(256) void gs(const f4* __restrict__ x, f4* __restrict__ y, long n4) {
    const long stride = (long)gridDim.x * 256 * U;
    for (long i = (long)blockIdx.x * 256 * U + threadIdx.x; i < n4; i += stride) {
        f4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long k = i + (long)u * 256;
            v[u] = k < n4 ? ld<NTL>(x + k) : f4{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long k = i + (long)u * 256;
            if (k < n4) st<NTS>(y + k, v[u]);
        }
    }
}

template <int U, int NTL, int NTS>
__global__ __launch_bounds__(256) void chunk(const f4* __restrict__ x, f4* __restrict__ y, long n4, int ch) {
    const long b0 = (long)blockIdx.x * ch;
    const long e = std::min(n4, b0 + ch);
    for (long i = b0 + threadIdx.x; i < e; i += 256 * U) {
        f4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long k = i + (long)u * 256;
            v[u] = k < e ? ld<NTL>(x + k) : f4{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long k = i + (long)u * 256;
            if (k < e) st<NTS>(y + k, v[u]);
        }
    }
}

template <int U>
__global__ __launch_bounds__(256) void rd(const f4* __restrict__ x, f4* __restrict__ y, long n4) {
    const long stride = (long)gridDim.x * 256 * U;
    f4 acc = {0, 0, 0, 0};
    for (long i = (long)blockIdx.x * 256 * U + threadIdx.x; i < n4; i += stride) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long k = i + (long)u * 256;
            if (k < n4) acc += x[k];
        }
    }
    if (acc[0] == 12345.f) y[threadIdx.x] = acc;
}

template <int NTS>
__global__ __launch_bounds__(256) void wr(f4* __restrict__ y, long n4) {
    const long stride = (long)gridDim.x * 256;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) st<NTS>(y + i, f4{1, 2, 3, 4});
}

// conv geometry: one wave = (image n, segment of RB rows); per row it reads the 16
// channel runs of the row (16 x W floats, W = 224: 56 float4 per channel -> lanes
// 0..55 per channel, 14 instructions of 64 lanes cover 16 x 56 = 896 float4) and
// stores the row read LAG rows earlier.  Data stays in VGPRs (ring of LAG+1 rows
// would be too big) -- instead the store writes the freshly loaded row at the
// output position of row r - LAG, which has the same traffic shape.
template <int NTS>
__global__ __launch_bounds__(256) void planes(const float* __restrict__ x, float* __restrict__ y, int N, int C,
                                              int H, int W, int RB, int lag) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nseg = (H + RB - 1) / RB;
    const int item = blockIdx.x * 4 + wave;
    if (item >= N * nseg) return;
    const int seg = item % nseg, n = item / nseg;
    const long plane = (long)H * W;
    const float* xn = x + (long)n * C * plane;
    float* yn = y + (long)n * C * plane;
    const int W4 = W / 4;
    const int per = C * W4;  // float4 per row
    const int r0 = seg * RB, r1 = std::min(H, r0 + RB);
    for (int r = r0; r < r1 + lag; ++r) {
        f4 v[14];
#pragma unroll
        for (int i = 0; i < 14; ++i) {
            const int e = i * 64 + lane;
            const int c = e / W4, q4 = e % W4;
            v[i] = (r < r1 && e < per) ? *reinterpret_cast<const f4*>(xn + c * plane + (long)r * W + 4 * q4)
                                       : f4{0, 0, 0, 0};
        }
        const int ro = r - lag;
        if (ro >= r0) {
#pragma unroll
            for (int i = 0; i < 14; ++i) {
                const int e = i * 64 + lane;
                const int c = e / W4, q4 = e % W4;
                if (e < per) st<NTS>(reinterpret_cast<f4*>(yn + c * plane + (long)ro * W + 4 * q4), v[i]);
            }
        }
    }
}


// planes with RPL image rows per step: a channel's RPL consecutive rows are one contiguous
// run of RPL x W floats, so a step reads C runs of RPL x W x 4 bytes (and writes as many
// LAG rows later) instead of C runs of one row.  C x RPL x W / 4 <= 64 x 14 x RPL float4.
template <int RPL, int NTL, int NTS>
__global__ __launch_bounds__(256) void planes_rpl(const float* __restrict__ x, float* __restrict__ y, int N, int C,
                                                  int H, int W, int RB, int lag, int pad, int skew) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nseg = (H + RB - 1) / RB;
    const int item = blockIdx.x * 4 + wave;
    if (item >= N * nseg) return;
    int seg = item % nseg;
    const int n = item / nseg;
    if (skew) seg = (seg + n) % nseg;  // concurrent blocks of different images at different rows
    const long plane = (long)H * W + pad;  // pad: an artificial channel-plane stride
    const float* xn = x + (long)n * C * plane;
    float* yn = y + (long)n * C * plane;
    const int RW4 = RPL * W / 4;  // float4 per channel run
    const int per = C * RW4;
    const int r0 = seg * RB, r1 = std::min(H, r0 + RB);
    for (int r = r0; r < r1 + lag; r += RPL) {
        f4 v[14 * RPL];
#pragma unroll
        for (int i = 0; i < 14 * RPL; ++i) {
            const int e = i * 64 + lane;
            const int c = e / RW4, q4 = e % RW4;
            const long off = c * plane + (long)r * W + 4 * q4;
            v[i] = (r < r1 && e < per && off < c * plane + (long)H * W) ? ld<NTL>(reinterpret_cast<const f4*>(xn + off))
                                                                 : f4{0, 0, 0, 0};
        }
        const int ro = r - lag;
        if (ro >= r0) {
#pragma unroll
            for (int i = 0; i < 14 * RPL; ++i) {
                const int e = i * 64 + lane;
                const int c = e / RW4, q4 = e % RW4;
                const long off = c * plane + (long)ro * W + 4 * q4;
                if (e < per && off < c * plane + (long)H * W) st<NTS>(reinterpret_cast<f4*>(yn + off), v[i]);
            }
        }
    }
}


// ---- the conv's memory walk with no compute: LDS-DMA ring of PD rows, each landed
// row read back (ds_read_b128) and stored to the same position of y.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t mkrs(const void* p, uint32_t bytes) {
    const uintptr_t bp = reinterpret_cast<uintptr_t>(p);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)bp);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(bp >> 32));
    void* b = reinterpret_cast<void*>(((uintptr_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(b, (short)0, bytes, 0x00020000);
}
template <int NTL>
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t lds_addr) {
    if constexpr (NTL)
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %2, 0 offen nt lds"
                     ::"v"(voff), "s"(lds_addr), "s"(rs) : "memory");
    else
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %2, 0 offen lds"
                     ::"v"(voff), "s"(lds_addr), "s"(rs) : "memory");
}
template <int NTS>
__device__ __forceinline__ void st16(__amdgpu_buffer_rsrc_t rs, uint32_t vo, f4 v) {
    if constexpr (NTS)
        asm volatile("buffer_store_dwordx4 %0, %1, %2, 0 offen nt" ::"v"(v), "v"(vo), "s"(rs) : "memory");
    else
        asm volatile("buffer_store_dwordx4 %0, %1, %2, 0 offen" ::"v"(v), "v"(vo), "s"(rs) : "memory");
}
template <int N>
__device__ __forceinline__ void vmw() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// wave item = (image, segment of RB output rows, strip of SW columns); C = 16 channels;
// NI = C*SW/256 DMA instructions (1 KiB) per halo row; lane l of instruction i ->
// e = 64i + l: channel e / (SW/4), float4 column e % (SW/4).  BLK: a block of 4 waves
// owns (image, segment) and wave w the 4 channels 4w..4w+3 over the full width
// (SW = W; NI = 4, the last instruction part-masked); BAR: one s_barrier per row.
template <int SW, int PD, int NTL, int NTS, int BLK, int BAR, int HALO = 0, int LDSR = 0, int LDSW = 0>
__global__ __launch_bounds__(256) void ring(const float* __restrict__ x, float* __restrict__ y, int N, int H, int W,
                                            int RB) {
    constexpr int C = 16;
    constexpr int LPC = SW / 4;
    constexpr int NI = BLK ? (4 * LPC + 63) / 64 : C * LPC / 64;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nstrip = BLK ? 1 : (W + SW - 1) / SW, nseg = (H + RB - 1) / RB;
    int blk = blockIdx.x;
    blk = (blk & 7) * (int)(gridDim.x >> 3) + (blk >> 3);
    const int item = BLK ? blk : blk * 4 + wave;
    if (item >= N * nseg * nstrip) return;
    const int strip = item % nstrip, seg = (item / nstrip) % nseg, n = item / (nstrip * nseg);
    const uint32_t plane = (uint32_t)H * W;
    const __amdgpu_buffer_rsrc_t rx = mkrs(x + (int64_t)n * C * plane, C * plane * 4u);
    const __amdgpu_buffer_rsrc_t ry = mkrs(y + (int64_t)n * C * plane, C * plane * 4u);
    constexpr int SLOT = NI * 1024 + (HALO ? 256 : 0);
    unsigned char* slab = lds + wave * (PD * SLOT);
    const uint32_t slab_a = (uint32_t)(uintptr_t)slab;
    uint32_t voff[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const int e = 64 * i + lane;
        const int c = (BLK ? 4 * wave : 0) + e / LPC, q4 = e % LPC;
        const bool ok = (BLK ? e < 4 * LPC : true) && strip * SW + 4 * q4 < W;
        voff[i] = ok ? ((uint32_t)c * plane + (uint32_t)(strip * SW + 4 * q4)) * 4u : 0x7fffffffu;
    }
    const int r0 = seg * RB, rbe = min(RB, H - r0), nrows = rbe + 2;
    // HALO: the conv's halo-column DMA (one dword per lane, lanes 0..31: side x channel)
    const int hq = (lane >> 4) ? strip * SW + SW : strip * SW - 1;
    const uint32_t hoff = (lane < 32 && hq >= 0 && hq < W) ? ((uint32_t)(lane & 15) * plane + (uint32_t)hq) * 4u
                                                          : 0x7fffffffu;
    auto ldrow = [&](int sl, int j) __attribute__((always_inline)) {
        const int h = r0 - 1 + j;
        const bool ok = j < nrows && h >= 0 && h < H;
#pragma unroll
        for (int i = 0; i < NI; ++i)
            dma16<NTL>(rx, (ok && voff[i] != 0x7fffffffu) ? voff[i] + (uint32_t)h * W * 4u : 0x7fffffffu,
                       slab_a + (uint32_t)(sl * SLOT + i * 1024));
        if constexpr (HALO) {
            const uint32_t vo = (ok && hoff != 0x7fffffffu) ? hoff + (uint32_t)h * W * 4u : 0x7fffffffu;
            asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dword %0, %2, 0 offen lds"
                         ::"v"(vo), "s"(slab_a + (uint32_t)(sl * SLOT + NI * 1024)), "s"(rx) : "memory");
        }
    };
    for (int j = 0; j < PD; ++j) ldrow(j, j);
    int sl = 0;
    uint4 dummy = make_uint4(0u, 0u, 0u, 0u);
    // extra LDS traffic per step, like the conv's fragment reads (LDSR x ds_read_b128 over
    // a 4 KiB window past the ring) and split writes (LDSW x ds_write_b128)
    unsigned char* extra = lds + 4 * (PD * SLOT) + wave * 4096;
    for (int j = 0; j < nrows; ++j) {
        vmw<(PD - 1) * (2 * NI + HALO)>();
        if constexpr (BAR) __builtin_amdgcn_s_barrier();
        const int h = r0 - 1 + j;
        const bool st_ok = j >= 1 && j <= rbe;  // halo rows are loaded, not stored
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const f4 v = *reinterpret_cast<const f4*>(slab + sl * SLOT + i * 1024 + 16 * lane);
            st16<NTS>(ry, (st_ok && voff[i] != 0x7fffffffu) ? voff[i] + (uint32_t)h * W * 4u : 0x7fffffffu, v);
        }
        ldrow(sl, j + PD);
        sl = sl + 1 == PD ? 0 : sl + 1;
#pragma unroll
        for (int k = 0; k < LDSW; ++k)
            *reinterpret_cast<uint4*>(extra + ((16 * lane + 1024 * k) & 4095)) = make_uint4(j, k, lane, 0u);
#pragma unroll
        for (int k = 0; k < LDSR; ++k) {
            const uint4 v = *reinterpret_cast<const uint4*>(extra + ((16 * lane + 336 * k) & 4080));
            dummy.x ^= v.x; dummy.y += v.y; dummy.z ^= v.z; dummy.w += v.w;
            asm volatile("" : "+v"(dummy.x), "+v"(dummy.y), "+v"(dummy.z), "+v"(dummy.w));
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (dummy.x == 0x12345u) y[0] = (float)dummy.y;
}

static float time_it(hipEvent_t a, hipEvent_t b, int reps, const std::function<void()>& f) {
    std::vector<float> t;
    for (int i = 0; i < 3; ++i) f();
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(a));
        f();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main(int argc, char** argv) {
    const int N = 256, C = 16, H = 224, W = 224;
    const long nf = (long)N * C * H * W, n4 = nf / 4;
    const double bytes = nf * 4.0;
    const int reps = argc > 1 ? atoi(argv[1]) : 20;
    float *x, *y;
    const long nalloc = nf + nf / 8;  // room for the padded plane strides of mode 4 (<= 1024 floats per plane)
    CK(hipMalloc(&x, nalloc * 4));
    CK(hipMalloc(&y, nalloc * 4));
    CK(hipMemset(x, 0, nalloc * 4));
    CK(hipMemset(y, 0, nalloc * 4));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const f4* x4 = reinterpret_cast<const f4*>(x);
    f4* y4 = reinterpret_cast<f4*>(y);
    auto report = [&](const char* name, double ms, double mult) {
        printf("{\"probe\": \"%s\", \"ms\": %.4f, \"TBps\": %.3f}\n", name, ms, bytes * mult / ms / 1e9);
        fflush(stdout);
    };
    char nm[128];

    const int mode = argc > 2 ? atoi(argv[2]) : 0;
    if (mode == 4) {
        // rows per step: stage 1 (16 ch @224) and stage 2 (32 ch @112, same bytes per row step)
#define RPLP(R, L, S, CC, HH, RB, PAD, SK)                                                                              \
    {                                                                                                          \
        const int nseg = (HH + RB - 1) / RB;                                                                   \
        const int NN = (int)(nf / ((long)CC * HH * HH));                                                       \
        const int g = (NN * nseg + 3) / 4;                                                                     \
        float ms = time_it(a, b, reps, [&] {                                                                   \
            hipLaunchKernelGGL((planes_rpl<R, L, S>), dim3(g), dim3(256), 0, 0, x, y, NN, CC, HH, HH, RB, 2, PAD, SK); \
        });                                                                                                    \
        snprintf(nm, sizeof nm, "planes_C%d_H%d_RPL%d_ntl%d_nts%d_RB%d_pad%d_skew%d", CC, HH, R, L, S, RB, PAD, SK); \
        report(nm, ms, 2.0);                                                                                   \
    }
        for (int rep2 = 0; rep2 < 2; ++rep2) {
            {
                float ms = time_it(a, b, reps, [&] { hipLaunchKernelGGL((gs<4, 1, 1>), dim3(4096), dim3(256), 0, 0, x4, y4, n4); });
                report("gs_U4_ntl1_nts1_g4096", ms, 2.0);
            }
            RPLP(1, 1, 1, 16, 224, 28, 0, 0) RPLP(1, 1, 1, 16, 224, 28, 0, 1) RPLP(1, 1, 1, 16, 224, 28, 64, 0)
            RPLP(1, 1, 1, 16, 224, 28, 256, 0) RPLP(1, 1, 1, 16, 224, 28, 1024, 0) RPLP(1, 1, 1, 16, 224, 28, 1024, 1)
            RPLP(2, 1, 1, 16, 224, 28, 1024, 1) RPLP(1, 1, 1, 16, 224, 8, 0, 0) RPLP(1, 1, 1, 16, 224, 8, 64, 0)
            RPLP(1, 1, 1, 32, 112, 28, 0, 0) RPLP(1, 1, 1, 32, 112, 28, 0, 1) RPLP(1, 1, 1, 32, 112, 28, 64, 0)
            RPLP(1, 1, 1, 32, 112, 28, 1024, 0) RPLP(2, 1, 1, 32, 112, 28, 1024, 1)
        }
        CK(hipDeviceSynchronize());
        return 0;
    }
    if (mode == 3) {
#define RING3(R, WR)                                                                                           \
    {                                                                                                          \
        const int nseg = (H + 25 - 1) / 25;                                                                    \
        const int items = N * nseg * 7;                                                                        \
        const int g = ((items + 3) / 4 + 7) / 8 * 8;                                                           \
        const int ldsb = 38016;                                                                                \
        float ms = time_it(a, b, reps, [&] {                                                                   \
            hipLaunchKernelGGL((ring<32, 2, 0, 1, 0, 0, 1, R, WR>), dim3(g), dim3(256), ldsb, 0, x, y, N, H, W, 25); \
        });                                                                                                    \
        snprintf(nm, sizeof nm, "ring32_halo1_occ16_ldsr%d_ldsw%d", R, WR);                                   \
        report(nm, ms, 2.0);                                                                                   \
    }
        for (int rep2 = 0; rep2 < 2; ++rep2) {
            RING3(0, 0) RING3(6, 0) RING3(12, 0) RING3(18, 0) RING3(24, 0) RING3(0, 3) RING3(0, 6) RING3(18, 6)
            RING3(36, 0) RING3(18, 12)
        }
        CK(hipDeviceSynchronize());
        return 0;
    }
    if (mode == 2) {
#define RING2(PD, S, HALO, LDS, RB)                                                                           \
    {                                                                                                          \
        const int nseg = (H + RB - 1) / RB;                                                                    \
        const int items = N * nseg * 7;                                                                        \
        const int g = ((items + 3) / 4 + 7) / 8 * 8;                                                           \
        const int ldsb = std::max(LDS, 4 * PD * (2048 + (HALO ? 256 : 0)));                                    \
        float ms = time_it(a, b, reps, [&] {                                                                   \
            hipLaunchKernelGGL((ring<32, PD, 0, S, 0, 0, HALO>), dim3(g), dim3(256), ldsb, 0, x, y, N, H, W, RB); \
        });                                                                                                    \
        snprintf(nm, sizeof nm, "ring32_PD%d_nts%d_halo%d_lds%d_RB%d", PD, S, HALO, ldsb, RB);                 \
        report(nm, ms, 2.0);                                                                                   \
    }
        for (int rep2 = 0; rep2 < 2; ++rep2) {
            RING2(2, 1, 0, 0, 25) RING2(2, 1, 1, 0, 25) RING2(2, 1, 0, 38016, 25) RING2(2, 1, 1, 38016, 25)
            RING2(2, 0, 1, 38016, 25) RING2(3, 1, 1, 47232, 19) RING2(3, 0, 1, 47232, 19) RING2(6, 1, 1, 74880, 28)
            RING2(2, 1, 1, 38016, 14) RING2(2, 1, 0, 38016, 14)
        }
        CK(hipDeviceSynchronize());
        return 0;
    }
    if (mode == 1) {
#define RING(SW, PD, L, S, B, BAR, RB)                                                                         \
    {                                                                                                          \
        const int nstrip = B ? 1 : (W + SW - 1) / SW, nseg = (H + RB - 1) / RB;                                           \
        const int items = N * nseg * nstrip;                                                                   \
        const int g = ((B ? items : (items + 3) / 4) + 7) / 8 * 8;                                             \
        constexpr int NI = B ? (SW + 63) / 64 : 16 * SW / 256;                                                 \
        const int ldsb = 4 * PD * NI * 1024;                                                                   \
        float ms = time_it(a, b, reps, [&] {                                                                   \
            hipLaunchKernelGGL((ring<SW, PD, L, S, B, BAR>), dim3(g), dim3(256), ldsb, 0, x, y, N, H, W, RB); \
        });                                                                                                    \
        snprintf(nm, sizeof nm, "ring_SW%d_PD%d_ntl%d_nts%d_blk%d_bar%d_RB%d_lds%d", SW, PD, L, S, B, BAR, RB, ldsb); \
        report(nm, ms, 2.0);                                                                                   \
    }
        RING(32, 2, 0, 0, 0, 0, 25) RING(32, 2, 0, 1, 0, 0, 25) RING(32, 3, 0, 0, 0, 0, 25) RING(32, 3, 0, 1, 0, 0, 25)
        RING(32, 2, 1, 0, 0, 0, 25) RING(32, 2, 1, 1, 0, 0, 25) RING(32, 4, 0, 0, 0, 0, 25) RING(32, 4, 0, 1, 0, 0, 25)
        RING(32, 2, 0, 0, 0, 0, 14) RING(32, 3, 0, 0, 0, 0, 14) RING(32, 2, 0, 0, 0, 0, 56) RING(32, 3, 0, 0, 0, 0, 56)
        RING(64, 2, 0, 0, 0, 0, 25) RING(64, 2, 0, 1, 0, 0, 25) RING(64, 3, 0, 0, 0, 0, 25) RING(64, 2, 1, 1, 0, 0, 25)
        RING(112, 2, 0, 0, 0, 0, 25) RING(112, 2, 0, 1, 0, 0, 25) RING(112, 2, 1, 1, 0, 0, 25) RING(112, 2, 0, 0, 0, 0, 14)
        RING(224, 2, 0, 0, 1, 0, 14) RING(224, 2, 0, 1, 1, 0, 14) RING(224, 2, 1, 1, 1, 0, 14) RING(224, 3, 0, 0, 1, 0, 14)
        RING(224, 2, 0, 0, 1, 1, 14) RING(224, 3, 0, 0, 1, 1, 14) RING(224, 2, 0, 0, 1, 0, 28) RING(224, 3, 0, 0, 1, 0, 8)
        RING(224, 4, 0, 0, 1, 0, 8) RING(224, 4, 0, 1, 1, 0, 8) RING(224, 4, 1, 1, 1, 0, 8) RING(224, 3, 1, 1, 1, 0, 14)
        CK(hipDeviceSynchronize());
        return 0;
    }
#define GS(U, L, S, G)                                                                           \
    {                                                                                            \
        float ms = time_it(a, b, reps, [&] { hipLaunchKernelGGL((gs<U, L, S>), dim3(G), dim3(256), 0, 0, x4, y4, n4); }); \
        snprintf(nm, sizeof nm, "gs_U%d_ntl%d_nts%d_g%d", U, L, S, G);                         \
        report(nm, ms, 2.0);                                                                     \
    }
    for (int g : {1024, 2048, 4096, 8192}) {
        GS(1, 0, 0, g) GS(2, 0, 0, g) GS(4, 0, 0, g) GS(4, 0, 1, g) GS(4, 1, 1, g) GS(8, 0, 0, g) GS(8, 0, 1, g)
    }
#define CH(U, L, S, CHN)                                                                          \
    {                                                                                             \
        const int g = (int)((n4 + CHN - 1) / CHN);                                                \
        float ms = time_it(a, b, reps, [&] { hipLaunchKernelGGL((chunk<U, L, S>), dim3(g), dim3(256), 0, 0, x4, y4, n4, CHN); }); \
        snprintf(nm, sizeof nm, "chunk_U%d_ntl%d_nts%d_ch%d", U, L, S, CHN);                    \
        report(nm, ms, 2.0);                                                                      \
    }
    for (int chn : {1024, 4096, 16384, 65536}) {
        CH(4, 0, 0, chn) CH(4, 0, 1, chn) CH(8, 0, 0, chn) CH(8, 0, 1, chn) CH(8, 1, 1, chn)
    }
    for (int g : {2048, 4096}) {
        float ms = time_it(a, b, reps, [&] { hipLaunchKernelGGL((rd<4>), dim3(g), dim3(256), 0, 0, x4, y4, n4); });
        snprintf(nm, sizeof nm, "read_only_U4_g%d", g);
        report(nm, ms, 1.0);
        ms = time_it(a, b, reps, [&] { hipLaunchKernelGGL((rd<8>), dim3(g), dim3(256), 0, 0, x4, y4, n4); });
        snprintf(nm, sizeof nm, "read_only_U8_g%d", g);
        report(nm, ms, 1.0);
        ms = time_it(a, b, reps, [&] { hipLaunchKernelGGL((wr<0>), dim3(g), dim3(256), 0, 0, y4, n4); });
        snprintf(nm, sizeof nm, "write_only_g%d", g);
        report(nm, ms, 1.0);
        ms = time_it(a, b, reps, [&] { hipLaunchKernelGGL((wr<1>), dim3(g), dim3(256), 0, 0, y4, n4); });
        snprintf(nm, sizeof nm, "write_only_nt_g%d", g);
        report(nm, ms, 1.0);
    }
    for (int rb : {8, 14, 16, 28, 56}) {
        for (int nts : {0, 1}) {
            const int nseg = (H + rb - 1) / rb;
            const int g = (N * nseg + 3) / 4;
            float ms = time_it(a, b, reps, [&] {
                if (nts)
                    hipLaunchKernelGGL((planes<1>), dim3(g), dim3(256), 0, 0, x, y, N, C, H, W, rb, 2);
                else
                    hipLaunchKernelGGL((planes<0>), dim3(g), dim3(256), 0, 0, x, y, N, C, H, W, rb, 2);
            });
            snprintf(nm, sizeof nm, "planes_RB%d_nts%d", rb, nts);
            report(nm, ms, 2.0);
        }
    }
    CK(hipDeviceSynchronize());
    return 0;
}
