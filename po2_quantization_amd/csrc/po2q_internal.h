// Internal declarations shared by the po2q translation units (not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <string>

namespace po2q {

void set_error(const std::string& msg);

constexpr int kThreads = 256;          // 4 waves of 64
constexpr int kMaxPartials = 1024;     // absmax partials (blocks of the reduction pass)

// ---------------------------------------------------------------- quantizer --
// Number of partial-max slots the reduction pass uses for an n-element tensor.
int absmax_blocks(int64_t n);

// Pass 1: per-block max(|w|) as fp32 bit patterns (NaN-propagating) into partial[0..blocks).
hipError_t launch_absmax(const float* w, int64_t n, unsigned* partial, int blocks, hipStream_t s);

// Pass 2, plain output: out[i] = Q(w[i]) (reference elementwise semantics).
hipError_t launch_quantize_plain(const float* w, int64_t n, const unsigned* partial, int nparts,
                                 int bits, int fsr, int mode, float* out, hipStream_t s);

// Conv geometry and tiling plan (host-side, shared by workspace sizing and launch).
struct ConvPlan {
    // problem
    int N, C, H, W, K, R, S, sh, sw, ph, pw, dh, dw, groups;
    int P, Q, Cg, Kg;
    // kernel choice
    int kind;      // 0 = MFMA fp32 implicit GEMM, 1 = depthwise direct, 2 = bf16x3 MFMA
    int MI, NJ;    // 16-channel groups per block, 16-pixel groups per wave
    int TP, TQ, tilesP, tilesQ;  // output pixel tile
    int CC, nchunks, kblocks;    // channel chunk, #chunks, #output-channel blocks per group
    int HH, WW, WWp, PS;         // LDS halo tile dims / row stride / plane stride (floats)
    int steps;                   // MFMA steps per chunk = R*S*CC/4
    int64_t packed_floats;       // packed weight buffer (floats)
    size_t lds_bytes;
    int64_t blocks;
};

bool make_plan(ConvPlan& p, int64_t N, int64_t C, int64_t H, int64_t W, int64_t K, int64_t R,
               int64_t S, int64_t sh, int64_t sw, int64_t ph, int64_t pw, int64_t dh, int64_t dw,
               int64_t groups, int mode, int flags);

// Pack (and quantize unless mode == 0) the weight into the plan's layout.
hipError_t launch_pack_weights(const ConvPlan& p, const float* w, const unsigned* partial, int nparts,
                               int bits, int fsr, int mode, float* packed, hipStream_t s);

hipError_t launch_conv(const ConvPlan& p, const float* x, const float* packed, const float* bias,
                       float* y, hipStream_t s);

}  // namespace po2q
