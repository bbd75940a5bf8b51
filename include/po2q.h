/*
 * po2q — MI355X (gfx950) power-of-two quantized convolution, C ABI.
 *
 * The drop-in boundary for the reference's hot path (mschoenb97/po2_quantization):
 * plain pointers, sizes and a HIP stream handle; no torch types.  Every entry
 * point is asynchronous on `stream` (no host synchronisation, no allocation):
 * the caller owns every buffer, including the workspace whose size the
 * matching *_workspace_bytes() function returns.  All device pointers are
 * device-resident fp32, contiguous NCHW / [K, C/groups, R, S].
 *
 * Return value: PO2Q_OK (0) or a PO2Q_ERR_* code; po2q_last_error() then
 * holds a message (thread-local).  Invalid arguments are rejected before any
 * launch, so an error leaves every output untouched.
 */
#ifndef PO2Q_H_
#define PO2Q_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* quantizer selection — the reference's quantizer_dict keys (utils/quantizers.py:156-161)
 * plus "no quantizer" (QuantizedConv2d with quantize_fn=None, quantized_conv.py:37-38) */
enum po2q_mode { PO2Q_MODE_NONE = 0, PO2Q_MODE_PO2 = 1, PO2Q_MODE_PO2_PLUS = 2 };

/* conv arithmetic (flags of po2q_qconv2d_f32) */
enum po2q_precision {
    PO2Q_PREC_AUTO = 0,   /* BF16X3 when eligible (po2/po2+ weights, groups == 1), else FP32 */
    PO2Q_PREC_FP32 = 1,   /* fp32-input MFMA, exact fp32 fma chain (any weights) */
    PO2Q_PREC_BF16X3 = 2  /* bf16 MFMA on exact operands: weights Q(w)/scale = +-2^e, activations
                             split by truncation into hi+mid+lo bf16 (exact); fp32 accumulation.
                             PO2Q_ERR_UNSUPPORTED when not eligible. */
};

enum po2q_status {
    PO2Q_OK = 0,
    PO2Q_ERR_INVALID = 1,     /* bad shape / argument (reference: RuntimeError from torch) */
    PO2Q_ERR_UNSUPPORTED = 2, /* valid for the reference but not implemented here */
    PO2Q_ERR_WORKSPACE = 3,   /* workspace too small */
    PO2Q_ERR_HIP = 4          /* HIP runtime error at launch */
};

const char* po2q_version(void);
const char* po2q_last_error(void);

/*
 * PO2 / PO2+ weight quantizer.
 * Replaces PowerOfTwoQuantizer.forward      (utils/quantizers.py:19-32)
 *      and PowerOfTwoPlusQuantizer.forward  (utils/quantizers.py:39-52)
 * out[i] = 2^e_i * sign(w_i) * max|w|, e_i = clamp(round(log2|w_i/max|w||), fsr-2^(bits-1), fsr-1)
 * (po2+: round(log2(a/1.5)+0.5)), bit-exact with the reference incl. NaN/inf/±0.
 * n == 0 is rejected (the reference's torch.max raises on an empty tensor).
 * mode: PO2Q_MODE_PO2 or PO2Q_MODE_PO2_PLUS.  1 <= bits <= 16.
 */
size_t po2q_quantize_workspace_bytes(int64_t n);
int po2q_quantize_f32(const float* w, float* out, int64_t n, int bits, int fsr, int mode,
                      void* workspace, size_t workspace_bytes, void* stream);
/*
 * The same for fp64 and bf16 weights, in the weight's dtype as the reference computes it (its
 * torch ops keep the input dtype): fp64 with double arithmetic; bf16 (w, out as bf16 bit
 * patterns) with torch's bf16 arithmetic, every step in fp32 rounded to bf16.  Bit-exact with the
 * reference run on CPU in that dtype (decision tables measured from it,
 * tests/golden/gen_thresholds_dtypes.py).  Same workspace size function.
 */
int po2q_quantize_f64(const double* w, double* out, int64_t n, int bits, int fsr, int mode,
                      void* workspace, size_t workspace_bytes, void* stream);
int po2q_quantize_bf16(const uint16_t* w, uint16_t* out, int64_t n, int bits, int fsr, int mode,
                       void* workspace, size_t workspace_bytes, void* stream);

/*
 * Linear power-of-two quantizers lin / lin+ (per input channel = dim 1 of a 4-D weight).
 * Replaces LinearPowerOfTwoQuantizer.forward     (utils/quantizers.py:59-96)
 *      and LinearPowerOfTwoPlusQuantizer.forward (utils/quantizers.py:99-136):
 *   delta_c = (max_c - min_c) / (2^bits - 1), then num_iters least-squares refits of
 *   delta_c snapped to 2 ** round(log2(.)) (lin+: of sqrt(8/9) * delta_c);
 *   out = delta_c * clamp(round(w / delta_c), -(2^(bits-1) - 1), 2^(bits-1) - 1).
 * w, out [d0, d1, d2, d3] fp32 contiguous (may not alias).  Elementwise steps are the
 * reference's fp32 operations; the two refit sums are fp64 (deterministic).  A constant
 * channel (delta 0) or a NaN gives NaN, as in the reference.  Every d > 0 (the
 * reference's torch.max(dim) raises on an empty dim), 1 <= bits <= 16, num_iters >= 0,
 * plus 0 (lin) or 1 (lin+).  No workspace.
 */
int po2q_quantize_lin_f32(const float* w, float* out, int64_t d0, int64_t d1, int64_t d2, int64_t d3, int bits,
                          int num_iters, int plus, void* stream);

/*
 * Quantized 2-D convolution forward (quantize weight, then conv; NCHW fp32).
 * Replaces QuantizedConv2d.forward (models/quantized_conv.py:32-38), i.e.
 * F.conv2d(x, quantize_fn.apply(weight, bits), bias, stride, padding, dilation, groups);
 * mode PO2Q_MODE_NONE is the plain conv of quantize_fn=None (:37-38).
 * x [N, C, H, W], w [K, C/groups, R, S], bias [K] or NULL, y [N, K, P, Q] with
 * P = (H + 2*pad_h - dil_h*(R-1) - 1)/stride_h + 1 (likewise Q).
 * flags: one of enum po2q_precision.  The workspace size depends on every
 * argument of po2q_qconv2d_workspace_bytes (the plan is chosen from them); it
 * covers every plan po2q_qconv2d_autotune may select.
 */
size_t po2q_qconv2d_workspace_bytes(int64_t N, int64_t C, int64_t H, int64_t W,
                                    int64_t K, int64_t R, int64_t S,
                                    int64_t stride_h, int64_t stride_w, int64_t pad_h, int64_t pad_w,
                                    int64_t dil_h, int64_t dil_w, int64_t groups,
                                    int bits, int fsr, int mode, int flags);
int po2q_qconv2d_f32(const float* x, const float* w, const float* bias, float* y,
                     int64_t N, int64_t C, int64_t H, int64_t W,
                     int64_t K, int64_t R, int64_t S,
                     int64_t stride_h, int64_t stride_w, int64_t pad_h, int64_t pad_w,
                     int64_t dil_h, int64_t dil_w, int64_t groups,
                     int bits, int fsr, int mode, int flags,
                     void* workspace, size_t workspace_bytes, void* stream);

/*
 * Conv forward with its eval-mode epilogue fused into the launch:
 *   y = act((conv(x, Q(w)) + bias) * post_scale[k] + post_shift[k] + residual)
 * i.e. QuantizedConv2d.forward followed by the reference's eval BatchNorm (folded by
 * the caller into post_scale = gamma / sqrt(var + eps), post_shift = beta - mean *
 * post_scale), the residual add and the activation of its blocks:
 *   ResNet BasicBlock   relu(bn(conv(x)) [+ shortcut])   models/resnet.py:55-71
 *   MobileNetV2         relu6(bn(conv(x))) / bn(conv(x)) + x   models/mobilenet.py:32-33, 133-134
 *   MobileViT           silu(bn(conv(x)))                 models/mobile_vit.py:20-21, 225-227
 * post_scale / post_shift may be NULL (identity), residual may be NULL; residual is
 * [N, K, P, Q] like y and must not alias y (nor may x).  act: enum po2q_act.  Same
 * workspace as po2q_qconv2d_f32.  The row-streaming kernels apply the affine map and
 * the activation in their store epilogue (the C = K = 32 loader-wave plans the residual
 * add too); other plans and other residual adds run one extra elementwise pass over y.
 */
enum po2q_act { PO2Q_ACT_NONE = 0, PO2Q_ACT_RELU = 1, PO2Q_ACT_RELU6 = 2, PO2Q_ACT_SILU = 3 };

int po2q_qconv2d_fused_f32(const float* x, const float* w, const float* bias, float* y,
                           int64_t N, int64_t C, int64_t H, int64_t W,
                           int64_t K, int64_t R, int64_t S,
                           int64_t stride_h, int64_t stride_w, int64_t pad_h, int64_t pad_w,
                           int64_t dil_h, int64_t dil_w, int64_t groups,
                           int bits, int fsr, int mode, int flags,
                           const float* post_scale, const float* post_shift, const float* residual, int act,
                           void* workspace, size_t workspace_bytes, void* stream);

/*
 * Kernel autotuning, the counterpart of the reference's
 * torch.backends.cudnn.benchmark = True (train.py:33, test.py:31): times every
 * candidate plan for this problem on these buffers (synchronises the stream;
 * not allowed during graph capture), remembers the fastest for the process,
 * and leaves y = the chosen plan's result.  Later po2q_qconv2d_f32 /
 * po2q_qconv2d_describe calls with the same arguments use the tuned plan.
 * buf (may be NULL) receives the chosen plan's description.
 */
int po2q_qconv2d_autotune(const float* x, const float* w, const float* bias, float* y,
                          int64_t N, int64_t C, int64_t H, int64_t W,
                          int64_t K, int64_t R, int64_t S,
                          int64_t stride_h, int64_t stride_w, int64_t pad_h, int64_t pad_w,
                          int64_t dil_h, int64_t dil_w, int64_t groups,
                          int bits, int fsr, int mode, int flags,
                          void* workspace, size_t workspace_bytes, void* stream,
                          char* buf, size_t len);

/*
 * Plan enumeration (the counterpart of cuDNN's algorithm enumeration): returns
 * the number of candidate plans po2q_qconv2d_autotune times for these arguments
 * (>= 1; plan 0 is the heuristic default), or -status on invalid arguments, and
 * writes plan `index`'s description to buf when 0 <= index < count.
 * po2q_qconv2d_f32_plan runs candidate `index` (same contract as po2q_qconv2d_f32).
 */
int po2q_qconv2d_plans(int64_t N, int64_t C, int64_t H, int64_t W, int64_t K, int64_t R, int64_t S,
                       int64_t stride_h, int64_t stride_w, int64_t pad_h, int64_t pad_w,
                       int64_t dil_h, int64_t dil_w, int64_t groups,
                       int bits, int fsr, int mode, int flags, int index, char* buf, size_t len);
int po2q_qconv2d_f32_plan(int index, const float* x, const float* w, const float* bias, float* y,
                          int64_t N, int64_t C, int64_t H, int64_t W,
                          int64_t K, int64_t R, int64_t S,
                          int64_t stride_h, int64_t stride_w, int64_t pad_h, int64_t pad_w,
                          int64_t dil_h, int64_t dil_w, int64_t groups,
                          int bits, int fsr, int mode, int flags,
                          void* workspace, size_t workspace_bytes, void* stream);

/*
 * po2q_qconv2d_f32 in two enqueues, so the weight quantize + pack can run on another
 * stream, ahead of (and overlapped with) earlier convolutions:
 *   po2q_qconv2d_pack_f32    quantizes w and packs it into `workspace` (x, y untouched)
 *   po2q_qconv2d_packed_f32  runs the conv from that workspace (w untouched)
 * Same arguments and workspace size as po2q_qconv2d_f32; `plan` is -1 for the plan
 * po2q_qconv2d_f32 would run (tuned or heuristic) or a candidate index (as
 * po2q_qconv2d_f32_plan) -- both calls must name the same plan.  Ordering between the
 * two (and against later writes of w / reuse of the workspace) is the caller's, e.g. HIP
 * events; on one stream the pair equals po2q_qconv2d_f32 bit for bit.
 */
int po2q_qconv2d_pack_f32(int plan, const float* w,
                          int64_t N, int64_t C, int64_t H, int64_t W,
                          int64_t K, int64_t R, int64_t S,
                          int64_t stride_h, int64_t stride_w, int64_t pad_h, int64_t pad_w,
                          int64_t dil_h, int64_t dil_w, int64_t groups,
                          int bits, int fsr, int mode, int flags,
                          void* workspace, size_t workspace_bytes, void* stream);
int po2q_qconv2d_packed_f32(int plan, const float* x, const float* bias, float* y,
                            int64_t N, int64_t C, int64_t H, int64_t W,
                            int64_t K, int64_t R, int64_t S,
                            int64_t stride_h, int64_t stride_w, int64_t pad_h, int64_t pad_w,
                            int64_t dil_h, int64_t dil_w, int64_t groups,
                            int bits, int fsr, int mode, int flags,
                            const void* workspace, size_t workspace_bytes, void* stream);

/*
 * Diagnostic: the plan po2q_qconv2d_f32 would run for these arguments, as a
 * NUL-terminated text ("kind=bf16x3 CC=16 NT=1 NJ=4 tile=8x32 ..."), written
 * to buf (truncated to len).  No reference counterpart; used by bench.py and
 * tests to name the kernel that was measured.
 */
int po2q_qconv2d_describe(int64_t N, int64_t C, int64_t H, int64_t W, int64_t K, int64_t R, int64_t S,
                          int64_t stride_h, int64_t stride_w, int64_t pad_h, int64_t pad_w,
                          int64_t dil_h, int64_t dil_w, int64_t groups,
                          int bits, int fsr, int mode, int flags, char* buf, size_t len);

/*
 * QAT backward, weight gradient: the gradient autograd takes through
 * F.conv2d(x, Q(w), ...) for w -- the straight-through estimator passes it unchanged
 * (utils/quantizers.py:34-36; train.py:79-91 runs loss.backward()):
 *   dw[k][c][r][s] = sum_{n,p,q} dy[n][k][p][q] * x[n][c][p*sh + r*dil_h - pad_h][q*sw + s*dil_w - pad_w]
 * fp32 MFMA (exact products, fp32 accumulation, a fixed summation order: deterministic).
 * groups == 1, R x S in {1x1, 3x3}; or depthwise (groups == C == K, the MobileNetV2 / MobileViT
 * 3x3 depthwise QuantizedConv2d, reference models/mobilenet.py:64-76; R, S <= 5) through an
 * fp32 per-channel reduction (fixed order); PO2Q_ERR_UNSUPPORTED otherwise (the caller falls back).
 * The input gradient needs no entry of its own: for stride 1 it is po2q_qconv2d_f32 of dy
 * with the weight transposed (K <-> C) and flipped, padding R - 1 - pad (Q is
 * permutation-equivariant, so the same PO2 weights result).
 */
size_t po2q_qconv2d_wgrad_workspace_bytes(int64_t N, int64_t C, int64_t H, int64_t W, int64_t K, int64_t R,
                                          int64_t S, int64_t stride_h, int64_t stride_w, int64_t pad_h,
                                          int64_t pad_w, int64_t dil_h, int64_t dil_w, int64_t groups);
int po2q_qconv2d_wgrad_f32(const float* x, const float* dy, float* dw,
                           int64_t N, int64_t C, int64_t H, int64_t W, int64_t K, int64_t R, int64_t S,
                           int64_t stride_h, int64_t stride_w, int64_t pad_h, int64_t pad_w,
                           int64_t dil_h, int64_t dil_w, int64_t groups,
                           void* workspace, size_t workspace_bytes, void* stream);

/*
 * Zero insertion for strided input gradients (QAT backward, reference train.py:79-91): the input
 * gradient of a stride-(sh, sw) conv is the stride-1 conv of dy with (s - 1) zeros between its
 * pixels, with the weight transposed (K <-> C per group) and flipped -- po2q_qconv2d_f32 on the
 * same PO2 weights.  dst [N, C, Hd, Wd]: dst[n][c][i][j] = src[n][c][i/sh][j/sw] where sh | i,
 * sw | j and the source pixel exists, else 0.  src [N, C, P, Q].
 */
int po2q_dilate_f32(const float* src, float* dst, int64_t N, int64_t C, int64_t P, int64_t Q,
                    int64_t stride_h, int64_t stride_w, int64_t Hd, int64_t Wd, void* stream);

/*
 * Two chained quantized convs in one launch (ResNet56 stage-1 BasicBlock, reference
 * models/resnet.py:55-71; each conv is QuantizedConv2d.forward, models/quantized_conv.py:
 * 32-38; stage 2 takes it too): 3x3 / stride 1 / pad 1, C -> C -> C channels with C = 16 or
 * 32, x [N,C,H,W], w1 / w2 [C,C,3,3] quantized with the same (bits, fsr, mode):
 *   h = act1((conv(x, Q(w1)) + bias1) * post_scale1 + post_shift1)
 *   y = act2((conv(h, Q(w2)) + bias2) * post_scale2 + post_shift2 + residual)
 * (the affine first, then the residual add, then the activation; a NULL residual adds nothing)
 * (every pointer but x, w1, w2, y may be NULL).  h never leaves the chip.  No workspace.
 * po2q_qconv2d_pair_f32 takes C in {16, 32}, W % 4 == 0, W <= 7 * 512 / C (224 for C = 16,
 * 112 for C = 32), mode po2 / po2+ with the exponent window inside bf16's range.
 * po2q_qconv2d_pair_supported: 1 when it takes the shape AND is the faster path (C = 16 with
 * W > 96, C = 32 with W > 48 -- PO2Q_PAIR_C32=0 turns C = 32 off; otherwise two single-conv
 * calls).
 */
int po2q_qconv2d_pair_supported(int64_t N, int64_t C, int64_t H, int64_t W, int bits, int fsr, int mode);
int po2q_qconv2d_pair_f32(const float* x, const float* w1, const float* w2, float* y,
                          int64_t N, int64_t C, int64_t H, int64_t W, int bits, int fsr, int mode,
                          const float* bias1, const float* bias2,
                          const float* post_scale1, const float* post_shift1, int act1,
                          const float* post_scale2, const float* post_shift2, const float* residual, int act2,
                          void* stream);

/*
 * A chain of n_layers quantized 3x3 / stride-1 / pad-1 C -> C convs on small images in ONE
 * launch: the stride-1 run of a ResNet stage at CIFAR size -- consecutive
 * QuantizedConv2d.forward calls (models/quantized_conv.py:32-38) as models/resnet.py:55-71 /
 * 25-50 chain them, each with its BasicBlock's eval BN / ReLU / identity shortcut:
 *   a_0 = x;  a_{l+1} = act[l]((conv(a_l, Q(w[l])) + bias[l]) * post_scale[l] + post_shift[l]
 *                              (+ a_{res_from[l]} when res_from[l] >= 0));  y = a_{n_layers}
 * w, bias, post_scale, post_shift: host arrays of n_layers DEVICE pointers (the three epilogue
 * arrays, and any entry of them, may be NULL: skipped); act, res_from: host arrays (NULL: none;
 * res_from[l] in [-1, l], the residual is layer res_from[l]'s input).  Every weight is
 * [C, C, 3, 3], quantized with its own max|w| and the same (bits, fsr, mode).
 * One block per image runs every layer with the activation resident in LDS (only x is read and
 * y written); the weights are quantized + packed by batched launches first (the workspace holds
 * the packs).  The residual sources are held one at a time: two layers adding DIFFERENT sources
 * must not overlap (source <= the earlier user) -- the BasicBlock pattern [-1, 0, -1, 2, ...] and
 * any chain without residuals qualify.  Takes C in {16, 32, 64}, W % 4 == 0,
 * 1 <= n_layers <= PO2Q_CHAIN_MAX_LAYERS, (H + 2)(W + 2) 6C bytes <= 160 KiB and H * W <= 1024
 * (C = 16), 256 (C = 32), 128 (C = 64) -- ResNet's CIFAR stages --, mode po2 / po2+ with the
 * exponent window inside bf16's range.
 */
#define PO2Q_CHAIN_MAX_LAYERS 24
int po2q_qconv2d_chain_supported(int64_t N, int64_t C, int64_t H, int64_t W, int n_layers, int bits, int fsr,
                                 int mode);
size_t po2q_qconv2d_chain_workspace_bytes(int64_t N, int64_t C, int64_t H, int64_t W, int n_layers);
int po2q_qconv2d_chain_f32(const float* x, const float* const* w, const float* const* bias,
                           const float* const* post_scale, const float* const* post_shift, const int* act,
                           const int* res_from, int n_layers, int64_t N, int64_t C, int64_t H, int64_t W, int bits,
                           int fsr, int mode, float* y, void* workspace, size_t workspace_bytes, void* stream);

/*
 * The stride-2 transition of a ResNet56 stage (reference models/resnet.py:55-71 with the
 * projection shortcut: conv1 = QuantizedConv2d(C, 2C, 3, stride 2, padding 1) and
 * downsample.0 = QuantizedConv2d(C, 2C, 1, stride 2, padding 0), both
 * QuantizedConv2d.forward, models/quantized_conv.py:32-38, on the same x) in one launch:
 *   y   = act((conv3x3_s2(x, Q(w)))   * post_scale    + post_shift)
 *   yds =     conv1x1_s2(x, Q(wds))   * post_scale_ds + post_shift_ds
 * x [N, C, H, W], w [2C, C, 3, 3], wds [2C, C, 1, 1] (each quantized with its own max|w|,
 * the same bits / fsr / mode), y and yds [N, 2C, P, Q]; x is read once for both.  Every
 * epilogue pointer may be NULL.  C = 16 or 32, W % 4 == 0, po2 / po2+; no workspace.
 * po2q_qconv2d_s2ds_supported: 1 when the shape takes it AND it is the faster path (W >= 96;
 * on CIFAR-size rows two launches are faster).
 */
int po2q_qconv2d_s2ds_supported(int64_t N, int64_t C, int64_t H, int64_t W, int bits, int fsr, int mode);
int po2q_qconv2d_s2ds_f32(const float* x, const float* w, const float* wds, float* y, float* yds,
                          int64_t N, int64_t C, int64_t H, int64_t W, int bits, int fsr, int mode,
                          const float* post_scale, const float* post_shift, int act,
                          const float* post_scale_ds, const float* post_shift_ds, void* stream);

/*
 * Plan handles: a conv problem resolved ONCE to its kernel plan (the tuned plan when
 * po2q_qconv2d_autotune has measured it in this process, else the heuristic one; or
 * candidate `index` >= 0 of po2q_qconv2d_plans), so a framework binding that caches the
 * handle per problem pays no planning cost per call.  The PyTorch extension
 * (po2_quantization_amd/csrc/po2q_torch.cpp: torch.ops.po2q.*) keeps one per shape key.
 *   po2q_qconv2d_plan_create            resolve (same arguments as po2q_qconv2d_f32 + index)
 *   po2q_qconv2d_plan_workspace_bytes   the workspace THIS plan needs
 *   po2q_qconv2d_plan_run               quantize + conv (+ the fused epilogue of
 *                                       po2q_qconv2d_fused_f32: post_scale / post_shift /
 *                                       residual may be NULL, act PO2Q_ACT_*) on `stream`
 * Handles are immutable after creation; run may be called concurrently on one handle.
 * Replaces per call: QuantizedConv2d.forward (models/quantized_conv.py:32-38).
 */
typedef struct po2q_conv_plan po2q_conv_plan;
int po2q_qconv2d_plan_create(po2q_conv_plan** out, int index,
                             int64_t N, int64_t C, int64_t H, int64_t W,
                             int64_t K, int64_t R, int64_t S,
                             int64_t stride_h, int64_t stride_w, int64_t pad_h, int64_t pad_w,
                             int64_t dil_h, int64_t dil_w, int64_t groups,
                             int bits, int fsr, int mode, int flags);
size_t po2q_qconv2d_plan_workspace_bytes(const po2q_conv_plan* plan);
int po2q_qconv2d_plan_run(const po2q_conv_plan* plan, const float* x, const float* w, const float* bias, float* y,
                          const float* post_scale, const float* post_shift, const float* residual, int act,
                          void* workspace, size_t workspace_bytes, void* stream);
int po2q_qconv2d_plan_describe(const po2q_conv_plan* plan, char* buf, size_t len);
void po2q_qconv2d_plan_destroy(po2q_conv_plan* plan);

/*
 * The per-layer weight quantize + pack of a whole forward in one go (each layer's
 * QuantizedConv2d.forward quantizes its weight, models/quantized_conv.py:32-38): for every
 * plans[i] whose kernel does not stage its weight itself, quantize + pack w[i] into
 * workspace[i] (>= po2q_qconv2d_plan_workspace_bytes) -- the bf16x3 packs in
 * ceil(n / 36) launches instead of n.  po2q_qconv2d_plan_run_packed then runs plan's conv
 * from that workspace (w is read only by plans that stage their weight in-kernel); on one
 * stream the pair equals po2q_qconv2d_plan_run bit for bit.  The plans may differ in bits /
 * fsr / mode; depthwise plans join the batched launches too (their plain quantized copy).
 * po2q_qconv2d_plan_packs_weight: 1 when plan's conv reads a packed workspace (a pack
 * launch is due before po2q_qconv2d_plan_run_packed), 0 when the kernel stages the weight
 * itself or reads it as given (nothing to batch), < 0 on error.
 */
int po2q_qconv2d_plan_pack_batch(int n, const po2q_conv_plan* const* plans, const float* const* w,
                                 void* const* workspace, const size_t* workspace_bytes, void* stream);
int po2q_qconv2d_plan_packs_weight(const po2q_conv_plan* plan);
int po2q_qconv2d_plan_run_packed(const po2q_conv_plan* plan, const float* x, const float* w, const float* bias,
                                 float* y, const float* post_scale, const float* post_shift,
                                 const float* residual, int act, const void* workspace,
                                 size_t workspace_bytes, void* stream);

/*
 * One whole inverted-residual block in one launch (reference models/mobilenet.py:53-134,
 * InvertedResidual.forward :133-134; MobileViT's MV2Block, models/mobile_vit.py:131-239):
 *   h = act1(conv(x, Q(We)) * ps1 + pb1)                      [expand; skipped when expand == NULL: h = x]
 *   d = act2(dwconv3x3(h, Q(Wd), stride, pad 1) * ps2 + pb2)
 *   y = act3(conv(d, Q(Wp)) * ps3 + pb3 + residual)          [residual optional: the identity shortcut]
 * with the hidden activations h and d kept on chip.  expand / depthwise / project are the three
 * layers' plan handles (po2q_qconv2d_plan_create: the pointwise plans must be the bf16x3
 * pointwise kernel's, candidate index 0 of a 1x1 conv; the depthwise one a 3x3 pad-1 depthwise
 * conv) and ws_* their workspaces with the weights already staged (po2q_qconv2d_plan_pack_batch),
 * so Q(W) is recomputed by that pack in every forward as the reference does.  The layers are
 * bias-free (bias=False in the reference); ps / pb are the folded eval BatchNorms (NULL: 1 / 0).
 * Arithmetic: the pointwise plans' exact bf16x3 MFMA products and epilogue, the depthwise plan's
 * fp32 FMAs -- the layer chain's result up to the pointwise k-split summation order.
 * po2q_qconv2d_ir_supported: 1 when the three plans chain and a block geometry fits, 0 when not
 * (po2q_last_error() says why; run the three layers instead), < 0 on a bad argument.
 * po2q_qconv2d_ir_shape_supported: the same geometry test from the shapes alone (before any plan
 * exists): 1 when the block kernel takes it by default -- the small-image kernel at 3x3 / 4x4 images
 * (PO2Q_IR_SMALL=1: every image of <= 16 pixels; PO2Q_IR_LARGE=1: the chunked kernel for larger
 * ones), where it measured faster than the three layer launches.
 */
int po2q_qconv2d_ir_supported(const po2q_conv_plan* expand, const po2q_conv_plan* depthwise,
                              const po2q_conv_plan* project);
int po2q_qconv2d_ir_shape_supported(int64_t N, int64_t Cin, int64_t H, int64_t W, int64_t Ch, int64_t Cout,
                                    int64_t stride, int expand);
int po2q_qconv2d_ir_f32(const float* x, float* y, const po2q_conv_plan* expand, const void* ws_e, size_t ws_e_bytes,
                        const po2q_conv_plan* depthwise, const void* ws_d, size_t ws_d_bytes,
                        const po2q_conv_plan* project, const void* ws_p, size_t ws_p_bytes, const float* ps1,
                        const float* pb1, int act1, const float* ps2, const float* pb2, int act2, const float* ps3,
                        const float* pb3, const float* residual, int act3, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* PO2Q_H_ */
