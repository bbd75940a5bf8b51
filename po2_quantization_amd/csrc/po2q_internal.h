// Internal declarations shared by the po2q translation units (not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace po2q {

void set_error(const std::string& msg);

constexpr int kThreads = 256;          // 4 waves of 64
constexpr int kMaxPartials = 1024;     // absmax partials (blocks of the reduction pass)
constexpr int64_t kFusedAbsmaxMax = 1 << 20;  // weights up to this size: absmax fused into the pack kernel

// ---------------------------------------------------------------- quantizer --
// Number of partial-max slots the reduction pass uses for an n-element tensor.
int absmax_blocks(int64_t n);

// Pass 1: per-block max(|w|) as fp32 bit patterns (NaN-propagating) into partial[0..blocks).
hipError_t launch_absmax(const float* w, int64_t n, unsigned* partial, int blocks, hipStream_t s);

// Pass 2, plain output: out[i] = Q(w[i]) (reference elementwise semantics).
hipError_t launch_quantize_plain(const float* w, int64_t n, const unsigned* partial, int nparts,
                                 int bits, int fsr, int mode, float* out, hipStream_t s);

// Conv kinds
enum ConvKind {
    KIND_MFMA_F32 = 0,
    KIND_DEPTHWISE = 1,
    KIND_BF16X3 = 2,
    KIND_BF16X3_DMA = 3,
    KIND_BF16X3_ROWS = 4,
    KIND_BF16X3_PW = 5,  // 1x1 / stride 1 GEMM kernel (po2q_conv_pw.hip)
    KIND_DIRECT_F32 = 6,  // unquantized 3-channel stems, direct fp32 (po2q_conv_f32s.hip)
    KIND_PW_F32 = 7,      // unquantized 1x1 convs, fp32 MFMA GEMM (po2q_conv_f32s.hip)
    KIND_BF16X3_IMG = 8   // 3x3 / stride 1, small images: the block's rows resident in LDS (po2q_conv_img.hip)
};

// Every kind whose weight is packed as exact bf16 +-2^e fragments + one fp32 scale.
inline bool is_bf16x3_kind(int kind) {
    return kind == KIND_BF16X3 || kind == KIND_BF16X3_DMA || kind == KIND_BF16X3_ROWS || kind == KIND_BF16X3_PW ||
           kind == KIND_BF16X3_IMG;
}

// Conv geometry and tiling plan (host-side, shared by workspace sizing and launch).
struct ConvPlan {
    // problem
    int N, C, H, W, K, R, S, sh, sw, ph, pw, dh, dw, groups;
    int P, Q, Cg, Kg;
    // kernel choice
    int kind;
    int MI, NJ;    // fp32: 16-channel groups per block / 16-pixel groups per wave; bf16x3: NJ = pixel groups per wave
    int NT;        // bf16x3: 16-wide output-channel tiles per wave (K block = 16*NT)
    int TP, TQ, tilesP, tilesQ;  // output pixel tile
    int CC, nchunks, kblocks;    // channel chunk, #chunks, #output-channel blocks per group
    int HH, WW, WWp, PS;         // LDS halo tile dims / row stride / plane stride (floats, fp32 kind)
    int steps;                   // MFMA k-steps per chunk
    int SB;                      // bf16x3: LDS bytes per halo pixel (per split plane)
    int plane;                   // bf16x3: bytes per split plane (halo + 16 B zero pad)
    int taps;                    // R*S
    int vrx;                     // bf16x3: row-reuse schedule, waves across (0 = generic k-step schedule)
    int pd;                      // bf16x3 register kernel: x prefetch distance in work items (1 or 2)
    int nts;                     // row kernel (vrx 0): non-temporal output stores
    int fp = 0;                  // row kernels: weights quantized + packed inside the conv (one launch)
    int dma_d0, dma_nck, dma_ni, dma_nw;  // bf16x3 DMA: window offset, 16-B chunks per halo row, DMAs per wave
    int dma_waves;                // bf16x3 DMA: waves per block (4 or 8)
    int dma_ov;                   // bf16x3 DMA: overlapped pipeline (split of item i+1 under the MFMAs of item i)
    int64_t packed_floats;       // packed weight buffer (4-byte words)
    size_t lds_bytes;
    int64_t blocks;
};

// Default plan for a conv: the autotuned plan when po2q_qconv2d_autotune has
// measured this problem in this process, else the planners' heuristic choice.
bool make_plan(ConvPlan& p, int64_t N, int64_t C, int64_t H, int64_t W, int64_t K, int64_t R,
               int64_t S, int64_t sh, int64_t sw, int64_t ph, int64_t pw, int64_t dh, int64_t dw,
               int64_t groups, int mode, int bits, int fsr, int flags);

// Every plan worth timing for this problem (heuristic default first); false on invalid input.
bool plan_candidates(std::vector<ConvPlan>& out, int64_t N, int64_t C, int64_t H, int64_t W, int64_t K,
                     int64_t R, int64_t S, int64_t sh, int64_t sw, int64_t ph, int64_t pw, int64_t dh,
                     int64_t dw, int64_t groups, int mode, int bits, int fsr, int flags);

// Autotune cache: the measured-best plan per problem key (process-wide, thread-safe).
void tuned_store(const ConvPlan& p, int mode, int bits, int fsr, int flags);

// Fused weight staging source (plan field fp): the raw weight and the quantizer's
// parameters; w == nullptr selects the pre-packed workspace path.
struct WQuant {
    const float* w = nullptr;  // [K, C, 3, 3] fp32
    int n = 0;                 // weight elements
    int lo = 0, hi = 0;        // exponent clamp window
    int mode = 0;              // 0 po2, 1 po2+ (threshold row)
};

// Stride-2 full-row kernel (po2q_conv_rows2.hip: 3x3 s2 C -> 2C, plan vrx = 5, fused staging).
// yds != NULL: the same launch also computes the block's 1x1 stride-2 shortcut with the weight
// qd into yds ([N, K, P, Q]; epilogue psd / pbd when epi), reading x once for both convs.
hipError_t launch_conv_rows2(const ConvPlan& p, const float* x, const float* bias, float* y, hipStream_t s,
                             const float* ps, const float* pb, int act, bool epi, const WQuant& q,
                             float* yds = nullptr, const WQuant& qd = WQuant{}, const float* psd = nullptr,
                             const float* pbd = nullptr);

struct PlanCand {
    double cost;  // planner heuristic, lower is better
    ConvPlan plan;
};

// bf16x3 register-staged candidates (po2q_conv_x3.hip), cost-ranked; empty if the
// shape / exponent range is not eligible.  `base` is a validated geometry.
void x3_candidates(const ConvPlan& base, int mode, int bits, int fsr, std::vector<PlanCand>& out);
bool plan_bf16x3(ConvPlan& p, int mode, int bits, int fsr);

// LDS-DMA pipelined bf16x3 candidates (po2q_conv_x3p.hip), cost-ranked; empty if not
// eligible.  Call only for problems x3_candidates accepts (same arithmetic).
void x3p_candidates(const ConvPlan& base, std::vector<PlanCand>& out);
bool plan_bf16x3_dma(ConvPlan& p);

// Row-streaming bf16x3 candidates (po2q_conv_rows.hip: 3x3 / stride 1 / C in {16, 32});
// empty if not eligible.
void rows_candidates(const ConvPlan& base, int mode, int bits, int fsr, std::vector<PlanCand>& out);

// Pointwise 1x1 / stride-1 candidates (po2q_conv_pw.hip), cost-ranked; empty if not eligible.
void pw_candidates(const ConvPlan& base, int mode, int bits, int fsr, std::vector<PlanCand>& out);
// Its launch, the eval epilogue (ps / pb / res may be NULL, act PO2Q_ACT_*) in the store.
hipError_t launch_conv_pw(const ConvPlan& p, const float* x, const uint16_t* packed, const float* scale,
                          const float* bias, float* y, const float* ps, const float* pb, const float* res, int act,
                          hipStream_t s);

// Small-image 3x3 / stride-1 candidates (po2q_conv_img.hip), cost-ranked; empty if not eligible.
void img_candidates(const ConvPlan& base, int mode, int bits, int fsr, std::vector<PlanCand>& out);
// Its launch (row-kernel pack layout), the eval epilogue (ps / pb / res may be NULL) in the store.
hipError_t launch_conv_img(const ConvPlan& p, const float* x, const uint16_t* packed, const float* scale,
                           const float* bias, float* y, const float* ps, const float* pb, const float* res, int act,
                           hipStream_t s);

// fp32 kernels for mode none (po2q_conv_f32s.hip): candidates (empty if not eligible) and the
// launch with the eval epilogue in the store; the weight is read as given (no pack).
void f32s_candidates(const ConvPlan& base, std::vector<PlanCand>& out);
hipError_t launch_conv_f32s(const ConvPlan& p, const float* x, const float* w, const float* bias, float* y,
                            const float* ps, const float* pb, const float* res, int act, hipStream_t s);

// Pack (and quantize unless mode == 0) the weight into the plan's layout.
hipError_t launch_pack_weights(const ConvPlan& p, const float* w, const unsigned* partial, int nparts,
                               int bits, int fsr, int mode, float* packed, hipStream_t s);

// bf16x3: quantize + pack weights as exact bf16 +-2^e fragments, write the
// scale multiplier to *scale_out.  nparts == 0: absmax is reduced in-kernel.
hipError_t launch_pack_bf16x3(const ConvPlan& p, const float* w, const unsigned* partial, int nparts,
                              int bits, int fsr, int mode, uint16_t* packed, float* scale_out,
                              hipStream_t s);

// One weight tensor of a batched pack: plan (a bf16x3 kind, or KIND_DEPTHWISE: the plain
// quantized fp32 copy), weight, destination (bf16 fragments / fp32 copy), scale slot (bf16x3).
struct PackReq {
    const ConvPlan* plan;
    const float* w;
    void* packed;
    float* scale;
    int bits, fsr, mode;
    unsigned* partial = nullptr;  // absmax_blocks(n) words of the plan's workspace (null: fused absmax only)
};
// whether a plan's weight staging can join a batched pack (quantized, fused absmax size,
// bf16x3 or depthwise kind)
bool pack_batchable(const ConvPlan& p, int mode);
// n weight tensors (pack_batchable plans, each with its own bits / fsr / mode) in ceil(n / 36) launches
hipError_t launch_pack_batch(int n, const PackReq* reqs, hipStream_t s);
// The same for n bf16x3 weight tensors with one (bits, fsr, mode).
hipError_t launch_pack_bf16x3_batch(int n, const ConvPlan* const* plans, const float* const* w,
                                    uint16_t* const* packed, float* const* scale_out, int bits, int fsr, int mode,
                                    hipStream_t s);

// Depthwise 3x3 LDS-halo kernel (po2q_conv_dw.hip): plan (kind KIND_DEPTHWISE, vrx 1) and launch
// with the fused epilogue (ps / pb / res may be NULL, act PO2Q_ACT_*).
bool dw3_plan(ConvPlan& p);
bool dw3_plan_ok(const ConvPlan& p);
hipError_t launch_conv_dw3(const ConvPlan& p, const float* x, const float* qw, const float* bias, float* y,
                           const float* ps, const float* pb, const float* res, int act, hipStream_t s);
hipError_t launch_conv(const ConvPlan& p, const float* x, const float* packed, const float* bias,
                       float* y, hipStream_t s);

hipError_t launch_conv_bf16x3(const ConvPlan& p, const float* x, const uint16_t* packed,
                              const float* scale, const float* bias, float* y, hipStream_t s);

hipError_t launch_conv_bf16x3_rows(const ConvPlan& p, const float* x, const uint16_t* packed,
                                   const float* scale, const float* bias, float* y, hipStream_t s,
                                   const WQuant& q = WQuant{});

hipError_t launch_conv_bf16x3_dma(const ConvPlan& p, const float* x, const uint16_t* packed,
                                  const float* scale, const float* bias, float* y, hipStream_t s);

// Fused inverted-residual block (po2q_conv_ir.hip): expand 1x1 -> depthwise 3x3 -> project 1x1 with
// eval BN / activations / identity residual, hidden activations in LDS.
struct IrPlan {
    int G, R, RI, nbands, CHK, P, PG, Po, HP, xs;
    size_t lds, off_hid, off_dpl, off_cw;
    int64_t blocks;
    int small = 0;     // 1: conv_ir_small (G images of <= 16 pixels in one MFMA tile, hidden slices per wave)
    int ntw = 0, tg = 0;  // small: output tiles per wave, wave groups over the output tiles
};
struct IrEpi {
    const float *ps1, *pb1, *ps2, *pb2, *ps3, *pb3;  // each optional (NULL)
    int act1, act2, act3;
    const float* res;  // residual [N, Cout, Ho, Wo] or NULL
};
bool ir_plan(IrPlan& ip, int64_t N, int64_t Cin, int64_t H, int64_t W, int64_t Ch, int64_t Cout, int64_t S,
             bool expand);
// we / we_scale: the expand layer's pointwise (KIND_BF16X3_PW) pack, NULL when there is no expand;
// wd: the depthwise plain quantized copy [Ch][9]; wp / wp_scale: the project layer's pointwise pack.
hipError_t launch_conv_ir(const IrPlan& ip, const float* x, float* y, int N, int Cin, int H, int W, int Ch, int Cout,
                          int S, const uint16_t* we, const float* we_scale, const float* wd, const uint16_t* wp,
                          const float* wp_scale, const IrEpi& e, hipStream_t s);

// The stage-2 conv pair (C = 32, 96 < W <= 128) as 4 waves x 32 columns with every weight in VGPRs
// (po2q_conv_pairw.hip); po2q_qconv2d_pair_f32 routes the shapes it takes there.
bool pairw_applicable(int64_t N, int64_t C, int64_t H, int64_t W);
hipError_t pairw_launch(const float* x, const float* w1, const float* w2, float* y, int64_t N, int64_t H,
                        int64_t W, int bits, int fsr, int mode, const float* bias1, const float* bias2,
                        const float* post_scale1, const float* post_shift1, int act1, const float* post_scale2,
                        const float* post_shift2, const float* residual, int act2, hipStream_t s);

// fp64 / bf16 (bit patterns) PO2 / PO2+ quantizer (po2q_quant_dtypes.hip): absmax partials
// (nparts = absmax_blocks(n) uint64 words), then the quantize pass.
template <typename T>
hipError_t launch_quantize_dt(const T* w, T* out, int64_t n, int bits, int fsr, int mode, uint64_t* partial,
                              int nparts, hipStream_t s);

// lin / lin+ quantizer (po2q_lin.hip): w, out [d0, d1, rs = d2*d3], one block per d1 channel
hipError_t launch_quantize_lin(const float* w, float* out, int d0, int d1, int rs, int bits, int num_iters, int plus,
                               hipStream_t s);

}  // namespace po2q
