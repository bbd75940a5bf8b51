// Elementwise conv epilogue over y [N, K, P*Q] (one HBM pass, float4 when aligned):
//   y = act(y * ps[k] + pb[k] + res)
// The part of po2q_qconv2d_fused_f32 (include/po2q.h) that a conv kernel did not fuse
// into its own store epilogue: the residual add of the reference's blocks
// (resnet.py:55-71 `out += shortcut; relu`, mobilenet.py:133-134 `x + conv(x)`) and,
// for plans without an epilogue, the folded eval BatchNorm and the activation.
#include <hip/hip_runtime.h>

#include "po2q_epi.h"

namespace po2q {

template <bool AFF, bool RES>
__global__ __launch_bounds__(kThreads) void epilogue_kernel(float* __restrict__ y, int64_t nvec, int PQ4, int K,
                                                            const float* __restrict__ ps,
                                                            const float* __restrict__ pb,
                                                            const float* __restrict__ res, int act) {
    // one float4 per thread and iteration; PQ % 4 == 0, so a float4 never straddles channels
    float4* y4 = reinterpret_cast<float4*>(y);
    const float4* r4 = reinterpret_cast<const float4*>(res);
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * kThreads) {
        const int k = (int)((i / PQ4) % K);
        float4 v = y4[i];
        if constexpr (AFF) {
            const float a = ps ? ps[k] : 1.0f, b = pb ? pb[k] : 0.0f;
            v.x = v.x * a + b; v.y = v.y * a + b; v.z = v.z * a + b; v.w = v.w * a + b;
        }
        if constexpr (RES) {
            const float4 r = r4[i];
            v.x += r.x; v.y += r.y; v.z += r.z; v.w += r.w;
        }
        v.x = epi_act(v.x, act); v.y = epi_act(v.y, act); v.z = epi_act(v.z, act); v.w = epi_act(v.w, act);
        y4[i] = v;
    }
}

template <bool AFF, bool RES>
__global__ __launch_bounds__(kThreads) void epilogue_kernel_scalar(float* __restrict__ y, int64_t n, int64_t PQ,
                                                                   int K, const float* __restrict__ ps,
                                                                   const float* __restrict__ pb,
                                                                   const float* __restrict__ res, int act) {
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kThreads) {
        const int k = (int)((i / PQ) % K);
        float v = y[i];
        if constexpr (AFF) v = v * (ps ? ps[k] : 1.0f) + (pb ? pb[k] : 0.0f);
        if constexpr (RES) v += res[i];
        y[i] = epi_act(v, act);
    }
}

template <bool AFF, bool RES>
static hipError_t launch_epi_t(float* y, int64_t N, int64_t K, int64_t PQ, const ConvEpi& e, hipStream_t s) {
    const int64_t n = N * K * PQ;
    const bool vec = PQ % 4 == 0 && ((reinterpret_cast<uintptr_t>(y) | reinterpret_cast<uintptr_t>(e.res)) & 15) == 0 &&
                     PQ / 4 <= INT32_MAX;
    const int64_t work = vec ? n / 4 : n;
    int64_t blocks = (work + kThreads - 1) / kThreads;
    blocks = blocks < 1 ? 1 : (blocks > 8192 ? 8192 : blocks);
    if (vec)
        hipLaunchKernelGGL((epilogue_kernel<AFF, RES>), dim3((unsigned)blocks), dim3(kThreads), 0, s, y, work,
                           (int)(PQ / 4), (int)K, e.ps, e.pb, e.res, e.act);
    else
        hipLaunchKernelGGL((epilogue_kernel_scalar<AFF, RES>), dim3((unsigned)blocks), dim3(kThreads), 0, s, y, n, PQ,
                           (int)K, e.ps, e.pb, e.res, e.act);
    return hipGetLastError();
}

hipError_t launch_epilogue(float* y, int64_t N, int64_t K, int64_t PQ, const ConvEpi& e, bool affine_done,
                           hipStream_t s) {
    const bool aff = !affine_done && (e.ps || e.pb);
    if (aff) return e.res ? launch_epi_t<true, true>(y, N, K, PQ, e, s) : launch_epi_t<true, false>(y, N, K, PQ, e, s);
    return e.res ? launch_epi_t<false, true>(y, N, K, PQ, e, s) : launch_epi_t<false, false>(y, N, K, PQ, e, s);
}

}  // namespace po2q
