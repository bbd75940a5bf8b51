// Fused conv epilogue (eval BatchNorm affine, residual add, activation): the
// po2q_qconv2d_fused_f32 entry point (include/po2q.h).  Not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "po2q_internal.h"

namespace po2q {

// y = act(v * ps[k] + pb[k] + res) with ps / pb / res optional (NULL).
struct ConvEpi {
    const float* ps;   // post_scale [K] or NULL
    const float* pb;   // post_shift [K] or NULL
    const float* res;  // residual [N, K, P, Q] or NULL
    int act;           // PO2Q_ACT_*
    bool any() const { return ps || pb || res || act != 0; }
};

// The activations of the reference's blocks (nn.ReLU, nn.ReLU6, nn.SiLU); NaN
// propagates as in torch (comparisons, not fmin/fmax).
__device__ __forceinline__ float epi_act(float v, int act) {
    if (act == 1) return v < 0.0f ? 0.0f : v;                                // relu
    if (act == 2) return v <= 0.0f ? 0.0f : (v >= 6.0f ? 6.0f : v);         // relu6 = hardtanh(0, 6)
    if (act == 3) return v / (1.0f + expf(-v));                              // silu
    return v;
}

// epi_act with the activation a compile-time constant: no per-value branch on a runtime act (a
// kernel dispatches its whole epilogue once per layer / launch instead).
template <int ACT>
__device__ __forceinline__ float epi_act_ct(float v) {
    static_assert(ACT >= 0 && ACT <= 3, "activation");
    return epi_act(v, ACT);
}

// Calls f(std::integral_constant<int, ACT>{}) for a runtime act in 0..3 (wave-uniform: one scalar
// branch per call site).
template <class F>
__device__ __forceinline__ void with_act(int act, F&& f) {
    switch (act) {
        case 1: f(std::integral_constant<int, 1>{}); break;
        case 2: f(std::integral_constant<int, 2>{}); break;
        case 3: f(std::integral_constant<int, 3>{}); break;
        default: f(std::integral_constant<int, 0>{}); break;
    }
}

// Row-streaming kernels with the affine map + activation in their store epilogue
// (po2q_conv_rows.hip / po2q_conv_rowsk.hip); the residual add in the kernel too where the
// plan can: rows_res_ok / launch_conv_rows_res (po2q_conv_rows.hip) cover the full-row
// plans, rowsk_res_ok / launch_conv_rowsk_res the C = 32 loader-wave and every C = 64 plan;
// any other plan leaves the residual to launch_epilogue.
bool rows_res_ok(const ConvPlan& p);
hipError_t launch_conv_rows_res(const ConvPlan& p, const float* x, const uint16_t* packed, const float* scale,
                                const float* bias, float* y, const float* ps, const float* pb, const float* res,
                                int act, hipStream_t s, const WQuant& q = WQuant{});
bool rowsk_res_ok(const ConvPlan& p);
hipError_t launch_conv_rowsk_res(const ConvPlan& p, const float* x, const uint16_t* packed, const float* scale,
                                 const float* bias, float* y, const float* ps, const float* pb, const float* res,
                                 int act, hipStream_t s, const WQuant& q = WQuant{});
hipError_t launch_conv_bf16x3_rows_epi(const ConvPlan& p, const float* x, const uint16_t* packed,
                                       const float* scale, const float* bias, float* y, const float* ps,
                                       const float* pb, int act, hipStream_t s, const WQuant& q = WQuant{});

// The one-output-per-lane depthwise kernel (po2q_conv.hip, KIND_DEPTHWISE vrx 0) with the epilogue
// in its store.
hipError_t launch_conv_depthwise_epi(const ConvPlan& p, const float* x, const float* packed, const float* bias, float* y,
                                     const float* ps, const float* pb, const float* res, int act, hipStream_t s);

// One elementwise pass over y [N, K, PQ]: y = act(y * ps[k] + pb[k] + res) (ps / pb
// skipped when affine_done).
hipError_t launch_epilogue(float* y, int64_t N, int64_t K, int64_t PQ, const ConvEpi& e, bool affine_done,
                           hipStream_t s);

}  // namespace po2q
