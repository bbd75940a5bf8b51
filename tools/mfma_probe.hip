// Issue cost of the bf16 MFMA shapes on one SIMD: v_mfma_f32_16x16x32_bf16 (the bf16x3
// kernels' instruction) against v_mfma_f32_16x16x16_bf16 (half the K: a candidate for
// C = 16's third tap, which now multiplies a zero half).  One wave per SIMD, 4 independent
// accumulators, cycles from s_memtime over a long back-to-back run.
//   hipcc --offload-arch=gfx950 -O3 -o tools/mfma_probe tools/mfma_probe.hip && tools/mfma_probe
#include <hip/hip_runtime.h>

#include <cstdio>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int kIters = 4096;

template <int KIND>
__global__ __launch_bounds__(256) void probe(float* out, long long* cyc) {
    const int lane = threadIdx.x & 63;
    bf16x8 a8, b8;
    bf16x4 a4, b4;
    for (int i = 0; i < 8; ++i) {
        a8[i] = (__bf16)(0.001f * (lane + i));
        b8[i] = (__bf16)(0.002f * (lane - i));
    }
    for (int i = 0; i < 4; ++i) {
        a4[i] = a8[i];
        b4[i] = b8[i];
    }
    floatx4 acc[4];
    for (int k = 0; k < 4; ++k) acc[k] = floatx4{0.f, 0.f, 0.f, 0.f};
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if constexpr (KIND == 0)
                acc[k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, b8, acc[k], 0, 0, 0);
            else
                acc[k] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, acc[k], 0, 0, 0);
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0.f;
    for (int k = 0; k < 4; ++k) s += acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (lane == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

int main() {
    float* out;
    long long* cyc;
    (void)hipMalloc(&out, 256 * 256 * 4);
    (void)hipMalloc(&cyc, 256 * 4 * 8);
    long long h[1024];
    for (int kind = 0; kind < 2; ++kind) {
        for (int rep = 0; rep < 3; ++rep) {
            hipEvent_t e0, e1;
            (void)hipEventCreate(&e0);
            (void)hipEventCreate(&e1);
            (void)hipEventRecord(e0, 0);
            if (kind == 0)
                hipLaunchKernelGGL(probe<0>, dim3(256), dim3(256), 0, 0, out, cyc);
            else
                hipLaunchKernelGGL(probe<1>, dim3(256), dim3(256), 0, 0, out, cyc);
            (void)hipEventRecord(e1, 0);
            (void)hipEventSynchronize(e1);
            float ms = 0.f;
            (void)hipEventElapsedTime(&ms, e0, e1);
            (void)hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
            double mean = 0;
            for (int i = 0; i < 1024; ++i) mean += (double)h[i];
            mean /= 1024;
            // s_memtime counts at the shader clock on gfx9
            printf("{\"mfma\": \"%s\", \"rep\": %d, \"ms\": %.4f, \"memtime_per_mfma\": %.2f, \"ns_per_mfma\": %.3f}\n",
                   kind == 0 ? "16x16x32_bf16" : "16x16x16_bf16", rep, ms, mean / (4.0 * kIters),
                   ms * 1e6 / (4.0 * kIters));
        }
    }
    return 0;
}
