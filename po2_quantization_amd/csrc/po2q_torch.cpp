// PyTorch-ROCm operator library for po2q: torch.ops.po2q.* registered through
// TORCH_LIBRARY on top of the C ABI (include/po2q.h, libpo2q.so).  Host C++ only -- every
// kernel lives in libpo2q.so; this file turns torch tensors into pointers, keeps one
// resolved plan handle + workspace size per conv problem, and launches on torch's current
// HIP stream.  Replaces the reference's call sites:
//   po2q::quantize       PowerOfTwoQuantizer / PowerOfTwoPlusQuantizer.forward
//                        (utils/quantizers.py:19-56), fp32 / fp64 / bf16 (the reference keeps the dtype)
//   po2q::quantize_lin   LinearPowerOfTwo(Plus)Quantizer.forward (utils/quantizers.py:59-136)
//   po2q::qconv2d        QuantizedConv2d.forward: F.conv2d(x, Q(w), bias, ...)
//                        (models/quantized_conv.py:32-38)
//   po2q::qconv2d_fused  the same + eval BatchNorm affine, residual add and activation of
//                        the blocks (resnet.py:55-71, mobilenet.py:32-33, mobile_vit.py:20-21)
//   po2q::qconv2d_pair   two chained C -> C 3x3 qconvs (C = 16 or 32) (+ BN / act between and after, residual)
//   po2q::qconv2d_s2ds   a stage's 3x3 stride-2 conv1 + 1x1 stride-2 shortcut on one read of x
//                        in one launch: a ResNet56 stage-1 BasicBlock (resnet.py:55-71)
//   po2q::conv_wgrad     the QAT backward's weight gradient (train.py:79-91 loss.backward();
//                        STE, utils/quantizers.py:34-36), dense and depthwise
//   po2q::dilate         zero insertion for the strided layers' input gradient
//   po2q::qconv2d_chain  a stage's stride-1 run of C -> C 3x3 qconvs (BasicBlocks at CIFAR size)
//                        in one launch (resnet.py:55-71 chained by :131-143)
//   po2q::qconv2d_pack_batch / po2q::qconv2d_packed
//                        the weight quantize of every QuantizedConv2d.forward of a model forward
//                        (quantized_conv.py:35) as batched launches, then each conv (+ epilogue)
//                        from its packed workspace
//   po2q::qconv2d_ir     a whole inverted-residual block (expand 1x1 -> depthwise 3x3 -> project
//                        1x1, BN / ReLU6 / identity shortcut) in one launch from the three layers'
//                        packed workspaces (mobilenet.py:53-134, mobile_vit.py:131-239)
// Meta kernels give the output shapes (FX / torch.compile tracing, fake tensors).
// Errors are TORCH_CHECK -> RuntimeError, as F.conv2d raises for bad arguments.
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/library.h>

#include <array>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "po2q.h"

namespace {

std::string last_error() {
    const char* e = po2q_last_error();
    return e ? std::string(e) : std::string("po2q: unknown error");
}

void check_hip_f32(const at::Tensor& t, const char* what) {
    TORCH_CHECK(t.is_cuda(), "po2q: ", what, " must be a HIP device tensor (got ", t.device(),
                "); the po2q ops have no CPU path");
    TORCH_CHECK(t.scalar_type() == at::kFloat, "po2q: ", what, " must be float32 (got ", t.scalar_type(), ")");
}

// PyTorch-ROCm reports HIP devices as device type "cuda" (masquerading): the guard and
// stream helpers of that scheme map them onto the HIP runtime
using DeviceGuard = at::hip::HIPGuardMasqueradingAsCUDA;

void* stream_of(const at::Tensor& t) {
    return reinterpret_cast<void*>(at::hip::getCurrentHIPStreamMasqueradingAsCUDA(t.device().index()).stream());
}

// ---- conv problem -> plan handle cache (process-wide, thread-safe) -----------------
using Key = std::array<int64_t, 20>;  // 14 geometry + bits, fsr, mode, precision, plan index, device

struct PlanEntry {
    po2q_conv_plan* plan = nullptr;
    size_t ws = 0;
    bool tuned = false;  // created after po2q_qconv2d_autotune measured this problem
    ~PlanEntry() { po2q_qconv2d_plan_destroy(plan); }
};

std::mutex g_mu;
std::map<Key, std::unique_ptr<PlanEntry>> g_plans;
std::vector<std::unique_ptr<PlanEntry>> g_retired;  // replaced by a tuned entry; kept alive

struct Geometry {
    std::array<int64_t, 14> g;  // N C H W K R S sh sw ph pw dh dw groups
    std::vector<int64_t> yshape;
};

int64_t pick(at::IntArrayRef v, int i, const char* what) {
    TORCH_CHECK(v.size() == 1 || v.size() == 2, "po2q: ", what, " must have 1 or 2 elements");
    return v.size() == 1 ? v[0] : v[i];
}

Geometry conv_geometry(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias,
                       at::IntArrayRef stride, at::IntArrayRef padding, at::IntArrayRef dilation, int64_t groups) {
    check_hip_f32(x, "input");
    check_hip_f32(w, "weight");
    TORCH_CHECK(x.dim() == 4 && w.dim() == 4, "po2q: expected 4-D input and weight, got ", x.dim(), "-D and ",
                w.dim(), "-D");
    TORCH_CHECK(x.device() == w.device(), "po2q: input and weight must be on the same device");
    if (bias.has_value()) {
        check_hip_f32(*bias, "bias");
        TORCH_CHECK(bias->device() == x.device(), "po2q: bias must be on the input's device");
        TORCH_CHECK(bias->numel() == w.size(0), "po2q: bias must have ", w.size(0), " elements");
    }
    TORCH_CHECK(groups > 0, "po2q: non-positive groups is not supported");
    TORCH_CHECK(w.size(1) * groups == x.size(1), "po2q: Given groups=", groups, ", weight of size ", w.sizes(),
                ", expected input", x.sizes(), " to have ", w.size(1) * groups, " channels, but got ", x.size(1),
                " channels instead");
    Geometry G;
    const int64_t sh = pick(stride, 0, "stride"), sw = pick(stride, 1, "stride");
    const int64_t ph = pick(padding, 0, "padding"), pw = pick(padding, 1, "padding");
    const int64_t dh = pick(dilation, 0, "dilation"), dw = pick(dilation, 1, "dilation");
    G.g = {x.size(0), x.size(1), x.size(2), x.size(3), w.size(0), w.size(2), w.size(3), sh, sw, ph, pw, dh, dw, groups};
    const int64_t P = (x.size(2) + 2 * ph - dh * (w.size(2) - 1) - 1) / sh + 1;
    const int64_t Q = (x.size(3) + 2 * pw - dw * (w.size(3) - 1) - 1) / sw + 1;
    G.yshape = {x.size(0), w.size(0), std::max<int64_t>(P, 0), std::max<int64_t>(Q, 0)};
    return G;
}

// The plan for this problem: candidate `plan` (>= 0), or the tuned / heuristic plan
// (-1); autotune != 0 measures every candidate once first (an untimed first call, as
// torch.backends.cudnn.benchmark does), writing y.
PlanEntry* plan_for(const Geometry& G, int64_t bits, int64_t fsr, int64_t mode, int64_t prec, int64_t plan,
                    bool autotune, const at::Tensor& x, const at::Tensor& w, const float* bias, at::Tensor& y,
                    bool& y_written) {
    Key k;
    for (int i = 0; i < 14; ++i) k[i] = G.g[i];
    k[14] = bits; k[15] = fsr; k[16] = mode; k[17] = prec; k[18] = plan; k[19] = x.device().index();
    std::lock_guard<std::mutex> lock(g_mu);
    auto it = g_plans.find(k);
    if (it != g_plans.end() && (it->second->tuned || !autotune || plan >= 0)) return it->second.get();
    const auto& g = G.g;
    if (autotune && plan < 0) {
        const size_t wsb = po2q_qconv2d_workspace_bytes(g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7], g[8], g[9],
                                                        g[10], g[11], g[12], g[13], (int)bits, (int)fsr, (int)mode,
                                                        (int)prec);
        TORCH_CHECK(wsb > 0, last_error());
        at::Tensor ws = at::empty({(int64_t)wsb}, x.options().dtype(at::kByte));
        char desc[512];
        const int st = po2q_qconv2d_autotune(x.data_ptr<float>(), w.data_ptr<float>(), bias, y.data_ptr<float>(),
                                             g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7], g[8], g[9], g[10], g[11],
                                             g[12], g[13], (int)bits, (int)fsr, (int)mode, (int)prec, ws.data_ptr(),
                                             wsb, stream_of(x), desc, sizeof desc);
        TORCH_CHECK(st == 0, last_error());
        y_written = true;
    }
    auto e = std::make_unique<PlanEntry>();
    const int st = po2q_qconv2d_plan_create(&e->plan, (int)plan, g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7], g[8],
                                            g[9], g[10], g[11], g[12], g[13], (int)bits, (int)fsr, (int)mode, (int)prec);
    TORCH_CHECK(st == 0, last_error());
    e->ws = po2q_qconv2d_plan_workspace_bytes(e->plan);
    e->tuned = autotune && plan < 0;
    PlanEntry* out = e.get();
    if (it != g_plans.end()) g_retired.push_back(std::move(it->second));
    g_plans[k] = std::move(e);
    return out;
}

// The plan qconv2d would run for this problem without autotuning (candidate `plan` >= 0, or
// the tuned / heuristic one), created on first use; host-only (no device access).
PlanEntry* plan_lookup(const std::array<int64_t, 14>& g, int64_t bits, int64_t fsr, int64_t mode, int64_t prec,
                       int64_t plan, int64_t dev) {
    Key k;
    for (int i = 0; i < 14; ++i) k[i] = g[i];
    k[14] = bits; k[15] = fsr; k[16] = mode; k[17] = prec; k[18] = plan; k[19] = dev;
    std::lock_guard<std::mutex> lock(g_mu);
    auto it = g_plans.find(k);
    if (it != g_plans.end()) return it->second.get();
    auto e = std::make_unique<PlanEntry>();
    const int st = po2q_qconv2d_plan_create(&e->plan, (int)plan, g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7], g[8],
                                            g[9], g[10], g[11], g[12], g[13], (int)bits, (int)fsr, (int)mode, (int)prec);
    TORCH_CHECK(st == 0, last_error());
    e->ws = po2q_qconv2d_plan_workspace_bytes(e->plan);
    PlanEntry* out = e.get();
    g_plans[k] = std::move(e);
    return out;
}

const float* opt_ptr(const c10::optional<at::Tensor>& t) { return t.has_value() ? t->data_ptr<float>() : nullptr; }

at::Tensor qconv2d_impl(const at::Tensor& x_, const at::Tensor& w_, const c10::optional<at::Tensor>& bias_,
                        at::IntArrayRef stride, at::IntArrayRef padding, at::IntArrayRef dilation, int64_t groups,
                        int64_t bits, int64_t mode, int64_t fsr, int64_t prec, int64_t plan, int64_t autotune,
                        const c10::optional<at::Tensor>& post_scale_, const c10::optional<at::Tensor>& post_shift_,
                        const c10::optional<at::Tensor>& residual_, int64_t act) {
    const Geometry G = conv_geometry(x_, w_, bias_, stride, padding, dilation, groups);
    const DeviceGuard guard(x_.device());
    const at::Tensor x = x_.contiguous(), w = w_.contiguous();
    c10::optional<at::Tensor> bias, ps, pb, res;
    if (bias_.has_value()) bias = bias_->contiguous();
    for (auto [src, dst, what] : {std::make_tuple(&post_scale_, &ps, "post_scale"),
                                  std::make_tuple(&post_shift_, &pb, "post_shift")}) {
        if (src->has_value()) {
            check_hip_f32(**src, what);
            TORCH_CHECK((*src)->device() == x.device(), "po2q: ", what, " must be on the input's device");
            TORCH_CHECK((*src)->numel() == G.yshape[1], "po2q: ", what, " must have ", G.yshape[1], " elements, got ",
                        (*src)->numel());
            *dst = (*src)->contiguous();
        }
    }
    if (residual_.has_value()) {
        check_hip_f32(*residual_, "residual");
        TORCH_CHECK(residual_->device() == x.device(), "po2q: residual must be on the input's device");
        TORCH_CHECK(residual_->sizes() == at::IntArrayRef(G.yshape), "po2q: residual shape ", residual_->sizes(),
                    " does not match the output ", at::IntArrayRef(G.yshape));
        res = residual_->contiguous();
    }
    at::Tensor y = at::empty(G.yshape, x.options());
    if (G.yshape[0] == 0) return y;  // an empty batch: torch's F.conv2d returns an empty output
    const bool epi = ps.has_value() || pb.has_value() || res.has_value() || act != 0;
    bool y_written = false;
    // autotuning writes y through the plain conv; with an epilogue the tuned plan runs again
    PlanEntry* e = plan_for(G, bits, fsr, mode, prec, plan, autotune != 0, x, w, opt_ptr(bias), y, y_written);
    if (y_written && !epi) return y;
    at::Tensor ws = at::empty({(int64_t)e->ws}, x.options().dtype(at::kByte));
    const int st = po2q_qconv2d_plan_run(e->plan, x.data_ptr<float>(), w.data_ptr<float>(), opt_ptr(bias),
                                         y.data_ptr<float>(), opt_ptr(ps), opt_ptr(pb), opt_ptr(res), (int)act,
                                         ws.data_ptr(), e->ws, stream_of(x));
    TORCH_CHECK(st == 0, last_error());
    return y;
}

at::Tensor qconv2d(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias,
                   at::IntArrayRef stride, at::IntArrayRef padding, at::IntArrayRef dilation, int64_t groups,
                   int64_t bits, int64_t mode, int64_t fsr, int64_t prec, int64_t plan, int64_t autotune) {
    return qconv2d_impl(x, w, bias, stride, padding, dilation, groups, bits, mode, fsr, prec, plan, autotune,
                        c10::nullopt, c10::nullopt, c10::nullopt, 0);
}

at::Tensor qconv2d_fused(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias,
                         at::IntArrayRef stride, at::IntArrayRef padding, at::IntArrayRef dilation, int64_t groups,
                         int64_t bits, int64_t mode, int64_t fsr, int64_t prec, int64_t plan, int64_t autotune,
                         const c10::optional<at::Tensor>& post_scale, const c10::optional<at::Tensor>& post_shift,
                         const c10::optional<at::Tensor>& residual, int64_t act) {
    TORCH_CHECK(act >= 0 && act <= 3, "po2q: unknown activation ", act);
    return qconv2d_impl(x, w, bias, stride, padding, dilation, groups, bits, mode, fsr, prec, plan, autotune,
                        post_scale, post_shift, residual, act);
}

at::Tensor quantize(const at::Tensor& w_, int64_t bits, int64_t mode, int64_t fsr) {
    TORCH_CHECK(w_.is_cuda(), "po2q: input must be a HIP device tensor (got ", w_.device(),
                "); the po2q ops have no CPU path");
    const auto dt = w_.scalar_type();
    TORCH_CHECK(dt == at::kFloat || dt == at::kDouble || dt == at::kBFloat16,
                "po2q: quantize takes float32, float64 or bfloat16 (got ", dt, ")");
    TORCH_CHECK(mode == 1 || mode == 2, "po2q: quantize() needs mode po2 (1) or po2+ (2)");
    const DeviceGuard guard(w_.device());
    const at::Tensor w = w_.contiguous();
    at::Tensor out = at::empty_like(w);
    const int64_t n = w.numel();
    at::Tensor ws = at::empty({(int64_t)std::max<size_t>(po2q_quantize_workspace_bytes(n), 256)},
                              w.options().dtype(at::kByte));
    int st;
    if (dt == at::kFloat)
        st = po2q_quantize_f32(w.data_ptr<float>(), out.data_ptr<float>(), n, (int)bits, (int)fsr, (int)mode,
                               ws.data_ptr(), ws.numel(), stream_of(w));
    else if (dt == at::kDouble)
        st = po2q_quantize_f64(w.data_ptr<double>(), out.data_ptr<double>(), n, (int)bits, (int)fsr, (int)mode,
                               ws.data_ptr(), ws.numel(), stream_of(w));
    else
        st = po2q_quantize_bf16(reinterpret_cast<const uint16_t*>(w.data_ptr()), reinterpret_cast<uint16_t*>(out.data_ptr()),
                                n, (int)bits, (int)fsr, (int)mode, ws.data_ptr(), ws.numel(), stream_of(w));
    TORCH_CHECK(st == 0, last_error());
    return out;
}

at::Tensor quantize_lin(const at::Tensor& w_, int64_t bits, int64_t num_iters, int64_t plus) {
    check_hip_f32(w_, "input");
    // the reference reduces dims 3, 2, 0 explicitly (torch.max(..., dim=3) ...)
    TORCH_CHECK(w_.dim() == 4, "po2q: the lin quantizers need a 4-D weight (got ", w_.dim(), " dims)");
    const DeviceGuard guard(w_.device());
    const at::Tensor w = w_.contiguous();
    at::Tensor out = at::empty_like(w);
    const int st = po2q_quantize_lin_f32(w.data_ptr<float>(), out.data_ptr<float>(), w.size(0), w.size(1), w.size(2),
                                         w.size(3), (int)bits, (int)num_iters, plus ? 1 : 0, stream_of(w));
    TORCH_CHECK(st == 0, last_error());
    return out;
}

// QAT backward: weight gradient (fp32 MFMA; see po2q_qconv2d_wgrad_f32)
at::Tensor conv_wgrad(const at::Tensor& x_, const at::Tensor& dy_, at::IntArrayRef wshape, at::IntArrayRef stride,
                      at::IntArrayRef padding, at::IntArrayRef dilation, int64_t groups) {
    check_hip_f32(x_, "input");
    check_hip_f32(dy_, "grad_output");
    TORCH_CHECK(x_.dim() == 4 && dy_.dim() == 4 && wshape.size() == 4, "po2q: wgrad: 4-D input, grad_output, weight");
    TORCH_CHECK(x_.device() == dy_.device(), "po2q: wgrad: input and grad_output on different devices");
    const DeviceGuard guard(x_.device());
    const at::Tensor x = x_.contiguous(), dy = dy_.contiguous();
    const int64_t sh = pick(stride, 0, "stride"), sw = pick(stride, 1, "stride");
    const int64_t ph = pick(padding, 0, "padding"), pw = pick(padding, 1, "padding");
    const int64_t dh = pick(dilation, 0, "dilation"), dw = pick(dilation, 1, "dilation");
    // the C ABI takes no dy / gw shapes: they must be the geometry's, or the kernel would read
    // past dy or write past gw
    TORCH_CHECK(groups >= 1 && wshape[0] > 0 && wshape[0] % groups == 0 && wshape[1] * groups == x.size(1),
                "po2q: wgrad: weight shape ", wshape, " with groups=", groups, " does not match input channels ",
                x.size(1));
    TORCH_CHECK(sh > 0 && sw > 0 && dh > 0 && dw > 0 && ph >= 0 && pw >= 0, "po2q: wgrad: bad stride / padding / dilation");
    const int64_t P = (x.size(2) + 2 * ph - dh * (wshape[2] - 1) - 1) / sh + 1;
    const int64_t Q = (x.size(3) + 2 * pw - dw * (wshape[3] - 1) - 1) / sw + 1;
    TORCH_CHECK(dy.size(0) == x.size(0) && dy.size(1) == wshape[0] && dy.size(2) == P && dy.size(3) == Q,
                "po2q: wgrad: grad_output shape ", dy.sizes(), " is not [", x.size(0), ", ", wshape[0], ", ", P, ", ",
                Q, "]");
    const size_t wsb = po2q_qconv2d_wgrad_workspace_bytes(x.size(0), x.size(1), x.size(2), x.size(3), wshape[0],
                                                          wshape[2], wshape[3], sh, sw, ph, pw, dh, dw, groups);
    TORCH_CHECK(wsb > 0, last_error());
    at::Tensor ws = at::empty({(int64_t)wsb}, x.options().dtype(at::kByte));
    at::Tensor gw = at::empty(wshape, x.options());
    const int st = po2q_qconv2d_wgrad_f32(x.data_ptr<float>(), dy.data_ptr<float>(), gw.data_ptr<float>(), x.size(0),
                                          x.size(1), x.size(2), x.size(3), wshape[0], wshape[2], wshape[3], sh, sw, ph,
                                          pw, dh, dw, groups, ws.data_ptr(), wsb, stream_of(x));
    TORCH_CHECK(st == 0, last_error());
    return gw;
}

// QAT backward: zero insertion for strided input gradients (po2q_dilate_f32)
at::Tensor dilate(const at::Tensor& x_, at::IntArrayRef stride, at::IntArrayRef size) {
    check_hip_f32(x_, "input");
    TORCH_CHECK(x_.dim() == 4, "po2q: dilate: 4-D input");
    const DeviceGuard guard(x_.device());
    const at::Tensor x = x_.contiguous();
    const int64_t sh = pick(stride, 0, "stride"), sw = pick(stride, 1, "stride");
    const int64_t Hd = pick(size, 0, "size"), Wd = pick(size, 1, "size");
    at::Tensor out = at::empty({x.size(0), x.size(1), Hd, Wd}, x.options());
    if (out.numel() == 0) return out;
    const int st = po2q_dilate_f32(x.data_ptr<float>(), out.data_ptr<float>(), x.size(0), x.size(1), x.size(2),
                                   x.size(3), sh, sw, Hd, Wd, stream_of(x));
    TORCH_CHECK(st == 0, last_error());
    return out;
}

// Two chained C -> C -> C 3x3 convs (C in {16, 32}) in one launch (po2q_qconv2d_pair_f32)
void check_vec(const c10::optional<at::Tensor>& t, const at::Tensor& x, int64_t n, const char* what) {
    if (!t.has_value()) return;
    check_hip_f32(*t, what);
    TORCH_CHECK(t->device() == x.device(), "po2q: ", what, " must be on the input's device");
    TORCH_CHECK(t->numel() == n, "po2q: ", what, " must have ", n, " elements, got ", t->numel());
}

at::Tensor qconv2d_pair(const at::Tensor& x_, const at::Tensor& w1_, const at::Tensor& w2_, int64_t bits, int64_t mode,
                        int64_t fsr, const c10::optional<at::Tensor>& bias1, const c10::optional<at::Tensor>& bias2,
                        const c10::optional<at::Tensor>& ps1, const c10::optional<at::Tensor>& pb1, int64_t act1,
                        const c10::optional<at::Tensor>& ps2, const c10::optional<at::Tensor>& pb2,
                        const c10::optional<at::Tensor>& residual, int64_t act2) {
    check_hip_f32(x_, "input");
    check_hip_f32(w1_, "weight1");
    check_hip_f32(w2_, "weight2");
    TORCH_CHECK(x_.dim() == 4 && w1_.dim() == 4 && w2_.dim() == 4, "po2q: pair: 4-D input and weights");
    TORCH_CHECK(w1_.sizes() == w2_.sizes() && w1_.size(0) == x_.size(1) && w1_.size(1) == x_.size(1) &&
                    w1_.size(2) == 3 && w1_.size(3) == 3,
                "po2q: pair: weights must both be [C, C, 3, 3] with C = the input's channels");
    TORCH_CHECK(w1_.device() == x_.device() && w2_.device() == x_.device(), "po2q: pair: tensors on one device");
    const int64_t C = x_.size(1);
    for (auto [t, what] : {std::make_pair(&bias1, "bias1"), std::make_pair(&bias2, "bias2"),
                           std::make_pair(&ps1, "post_scale1"), std::make_pair(&pb1, "post_shift1"),
                           std::make_pair(&ps2, "post_scale2"), std::make_pair(&pb2, "post_shift2")})
        check_vec(*t, x_, C, what);
    if (residual.has_value()) {
        check_hip_f32(*residual, "residual");
        TORCH_CHECK(residual->sizes() == x_.sizes() && residual->device() == x_.device(),
                    "po2q: pair: residual must match the input's shape and device");
    }
    const DeviceGuard guard(x_.device());
    const at::Tensor x = x_.contiguous(), w1 = w1_.contiguous(), w2 = w2_.contiguous();
    auto cont = [](const c10::optional<at::Tensor>& t) -> c10::optional<at::Tensor> {
        return t.has_value() ? c10::optional<at::Tensor>(t->contiguous()) : c10::nullopt;
    };
    const auto b1c = cont(bias1), b2c = cont(bias2), s1 = cont(ps1), t1 = cont(pb1), s2 = cont(ps2), t2 = cont(pb2),
               rc = cont(residual);
    at::Tensor y = at::empty_like(x);
    if (x.size(0) == 0) return y;
    const int st = po2q_qconv2d_pair_f32(x.data_ptr<float>(), w1.data_ptr<float>(), w2.data_ptr<float>(),
                                         y.data_ptr<float>(), x.size(0), C, x.size(2), x.size(3), (int)bits, (int)fsr,
                                         (int)mode, opt_ptr(b1c), opt_ptr(b2c), opt_ptr(s1), opt_ptr(t1), (int)act1,
                                         opt_ptr(s2), opt_ptr(t2), opt_ptr(rc), (int)act2, stream_of(x));
    TORCH_CHECK(st == 0, last_error());
    return y;
}

at::Tensor qconv2d_pair_meta(const at::Tensor& x, const at::Tensor&, const at::Tensor&, int64_t, int64_t, int64_t,
                             const c10::optional<at::Tensor>&, const c10::optional<at::Tensor>&,
                             const c10::optional<at::Tensor>&, const c10::optional<at::Tensor>&, int64_t,
                             const c10::optional<at::Tensor>&, const c10::optional<at::Tensor>&,
                             const c10::optional<at::Tensor>&, int64_t) {
    return at::empty_like(x);
}

// A stage's stride-2 3x3 conv and its 1x1 stride-2 shortcut in one launch (po2q_qconv2d_s2ds_f32)
std::tuple<at::Tensor, at::Tensor> qconv2d_s2ds(const at::Tensor& x_, const at::Tensor& w_, const at::Tensor& wds_,
                                                int64_t bits, int64_t mode, int64_t fsr,
                                                const c10::optional<at::Tensor>& ps, const c10::optional<at::Tensor>& pb,
                                                int64_t act, const c10::optional<at::Tensor>& psd,
                                                const c10::optional<at::Tensor>& pbd) {
    check_hip_f32(x_, "input");
    check_hip_f32(w_, "weight");
    check_hip_f32(wds_, "shortcut weight");
    TORCH_CHECK(x_.dim() == 4 && w_.dim() == 4 && wds_.dim() == 4, "po2q: s2ds: 4-D input and weights");
    const int64_t C = x_.size(1), K = 2 * C;
    TORCH_CHECK(w_.size(0) == K && w_.size(1) == C && w_.size(2) == 3 && w_.size(3) == 3,
                "po2q: s2ds: weight must be [2C, C, 3, 3]");
    TORCH_CHECK(wds_.size(0) == K && wds_.size(1) == C && wds_.size(2) == 1 && wds_.size(3) == 1,
                "po2q: s2ds: shortcut weight must be [2C, C, 1, 1]");
    TORCH_CHECK(w_.device() == x_.device() && wds_.device() == x_.device(), "po2q: s2ds: tensors on one device");
    for (auto [t, what] : {std::make_pair(&ps, "post_scale"), std::make_pair(&pb, "post_shift"),
                           std::make_pair(&psd, "post_scale_ds"), std::make_pair(&pbd, "post_shift_ds")})
        check_vec(*t, x_, K, what);
    const DeviceGuard guard(x_.device());
    const at::Tensor x = x_.contiguous(), w = w_.contiguous(), wds = wds_.contiguous();
    auto cont = [](const c10::optional<at::Tensor>& t) -> c10::optional<at::Tensor> {
        return t.has_value() ? c10::optional<at::Tensor>(t->contiguous()) : c10::nullopt;
    };
    const auto s1 = cont(ps), t1 = cont(pb), s2 = cont(psd), t2 = cont(pbd);
    const int64_t P = (x.size(2) - 1) / 2 + 1, Q = (x.size(3) - 1) / 2 + 1;
    at::Tensor y = at::empty({x.size(0), K, P, Q}, x.options());
    at::Tensor yds = at::empty({x.size(0), K, P, Q}, x.options());
    if (x.size(0) == 0) return {y, yds};
    const int st = po2q_qconv2d_s2ds_f32(x.data_ptr<float>(), w.data_ptr<float>(), wds.data_ptr<float>(),
                                         y.data_ptr<float>(), yds.data_ptr<float>(), x.size(0), C, x.size(2),
                                         x.size(3), (int)bits, (int)fsr, (int)mode, opt_ptr(s1), opt_ptr(t1), (int)act,
                                         opt_ptr(s2), opt_ptr(t2), stream_of(x));
    TORCH_CHECK(st == 0, last_error());
    return {y, yds};
}

std::tuple<at::Tensor, at::Tensor> qconv2d_s2ds_meta(const at::Tensor& x, const at::Tensor&, const at::Tensor&,
                                                     int64_t, int64_t, int64_t, const c10::optional<at::Tensor>&,
                                                     const c10::optional<at::Tensor>&, int64_t,
                                                     const c10::optional<at::Tensor>&,
                                                     const c10::optional<at::Tensor>&) {
    const int64_t P = (x.size(2) - 1) / 2 + 1, Q = (x.size(3) - 1) / 2 + 1;
    return {at::empty({x.size(0), 2 * x.size(1), P, Q}, x.options()),
            at::empty({x.size(0), 2 * x.size(1), P, Q}, x.options())};
}

// ---- Meta (shape-only) implementations ------------------------------------------
at::Tensor qconv2d_meta(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias,
                        at::IntArrayRef stride, at::IntArrayRef padding, at::IntArrayRef dilation, int64_t groups,
                        int64_t, int64_t, int64_t, int64_t, int64_t, int64_t) {
    TORCH_CHECK(x.dim() == 4 && w.dim() == 4, "po2q: expected 4-D input and weight");
    const int64_t P = (x.size(2) + 2 * pick(padding, 0, "padding") - pick(dilation, 0, "dilation") * (w.size(2) - 1) -
                       1) / pick(stride, 0, "stride") + 1;
    const int64_t Q = (x.size(3) + 2 * pick(padding, 1, "padding") - pick(dilation, 1, "dilation") * (w.size(3) - 1) -
                       1) / pick(stride, 1, "stride") + 1;
    return at::empty({x.size(0), w.size(0), std::max<int64_t>(P, 0), std::max<int64_t>(Q, 0)}, x.options());
}

at::Tensor qconv2d_fused_meta(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias,
                              at::IntArrayRef stride, at::IntArrayRef padding, at::IntArrayRef dilation, int64_t groups,
                              int64_t bits, int64_t mode, int64_t fsr, int64_t prec, int64_t plan, int64_t autotune,
                              const c10::optional<at::Tensor>&, const c10::optional<at::Tensor>&,
                              const c10::optional<at::Tensor>&, int64_t) {
    return qconv2d_meta(x, w, bias, stride, padding, dilation, groups, bits, mode, fsr, prec, plan, autotune);
}

at::Tensor same_meta(const at::Tensor& w, int64_t, int64_t, int64_t) { return at::empty_like(w); }

at::Tensor dilate_meta(const at::Tensor& x, at::IntArrayRef, at::IntArrayRef size) {
    return at::empty({x.size(0), x.size(1), pick(size, 0, "size"), pick(size, 1, "size")}, x.options());
}

at::Tensor conv_wgrad_meta(const at::Tensor& x, const at::Tensor&, at::IntArrayRef wshape, at::IntArrayRef,
                           at::IntArrayRef, at::IntArrayRef, int64_t) {
    return at::empty(wshape, x.options());
}

// ---- a stage's stride-1 chain of C -> C 3x3 qconvs in one launch (po2q_qconv2d_chain_f32) ----
// Empty epilogue / act / res_from lists mean "none"; otherwise each has one entry per weight.
at::Tensor qconv2d_chain(const at::Tensor& x_, at::TensorList weights, int64_t bits, int64_t mode, int64_t fsr,
                         const c10::List<c10::optional<at::Tensor>>& biases,
                         const c10::List<c10::optional<at::Tensor>>& post_scales,
                         const c10::List<c10::optional<at::Tensor>>& post_shifts, at::IntArrayRef acts,
                         at::IntArrayRef res_from) {
    check_hip_f32(x_, "input");
    TORCH_CHECK(x_.dim() == 4, "po2q: chain: 4-D input");
    const int64_t n = (int64_t)weights.size();
    TORCH_CHECK(n >= 1 && n <= PO2Q_CHAIN_MAX_LAYERS, "po2q: chain: 1 to ", PO2Q_CHAIN_MAX_LAYERS, " layers, got ", n);
    const int64_t C = x_.size(1);
    for (auto [len, what] : {std::make_pair((int64_t)biases.size(), "biases"),
                             std::make_pair((int64_t)post_scales.size(), "post_scales"),
                             std::make_pair((int64_t)post_shifts.size(), "post_shifts"),
                             std::make_pair((int64_t)acts.size(), "acts"),
                             std::make_pair((int64_t)res_from.size(), "res_from")})
        TORCH_CHECK(len == 0 || len == n, "po2q: chain: ", what, " must have one entry per weight (", n, ") or none, got ",
                    len);
    const DeviceGuard guard(x_.device());
    const at::Tensor x = x_.contiguous();
    std::vector<at::Tensor> keep;
    std::vector<const float*> wp(n), bp(n, nullptr), sp(n, nullptr), hp(n, nullptr);
    for (int64_t i = 0; i < n; ++i) {
        check_hip_f32(weights[i], "chain weight");
        TORCH_CHECK(weights[i].dim() == 4 && weights[i].size(0) == C && weights[i].size(1) == C &&
                        weights[i].size(2) == 3 && weights[i].size(3) == 3,
                    "po2q: chain weight ", i, " must be [", C, ", ", C, ", 3, 3], got ", weights[i].sizes());
        TORCH_CHECK(weights[i].device() == x.device(), "po2q: chain: tensors on one device");
        keep.push_back(weights[i].contiguous());
        wp[i] = keep.back().data_ptr<float>();
    }
    auto vecs = [&](const c10::List<c10::optional<at::Tensor>>& l, std::vector<const float*>& out, const char* what) {
        for (int64_t i = 0; i < (int64_t)l.size(); ++i) {
            const c10::optional<at::Tensor> t = l.get(i);
            if (!t.has_value()) continue;
            check_vec(t, x, C, what);
            keep.push_back(t->contiguous());
            out[i] = keep.back().data_ptr<float>();
        }
    };
    vecs(biases, bp, "chain bias");
    vecs(post_scales, sp, "chain post_scale");
    vecs(post_shifts, hp, "chain post_shift");
    std::vector<int> av(acts.begin(), acts.end()), rv(res_from.begin(), res_from.end());
    for (int a : av) TORCH_CHECK(a >= 0 && a <= 3, "po2q: chain: unknown activation ", a);
    at::Tensor y = at::empty_like(x);
    if (x.size(0) == 0) return y;
    // 0 for a geometry the chain does not take: the entry point then reports why
    const size_t wsb = std::max<size_t>(po2q_qconv2d_chain_workspace_bytes(x.size(0), C, x.size(2), x.size(3), (int)n), 256);
    at::Tensor ws = at::empty({(int64_t)wsb}, x.options().dtype(at::kByte));
    const int st = po2q_qconv2d_chain_f32(x.data_ptr<float>(), wp.data(), biases.size() ? bp.data() : nullptr,
                                          post_scales.size() ? sp.data() : nullptr,
                                          post_shifts.size() ? hp.data() : nullptr, av.empty() ? nullptr : av.data(),
                                          rv.empty() ? nullptr : rv.data(), (int)n, x.size(0), C, x.size(2), x.size(3),
                                          (int)bits, (int)fsr, (int)mode, y.data_ptr<float>(), ws.data_ptr(), wsb,
                                          stream_of(x));
    TORCH_CHECK(st == 0, last_error());
    return y;
}

at::Tensor qconv2d_chain_meta(const at::Tensor& x, at::TensorList, int64_t, int64_t, int64_t,
                              const c10::List<c10::optional<at::Tensor>>&, const c10::List<c10::optional<at::Tensor>>&,
                              const c10::List<c10::optional<at::Tensor>>&, at::IntArrayRef, at::IntArrayRef) {
    return at::empty_like(x);
}

// ---- batched weight staging of a forward: pack once, run each conv from its workspace ----
// geometry: 11 ints per layer (N C H W of the layer's input, stride h/w, padding h/w,
// dilation h/w, groups); plans: the plan index per layer (-1: tuned / heuristic).  Returns
// one byte workspace per layer (views of one allocation); a layer whose kernel stages its
// weight itself (or reads it as given) gets an empty workspace and runs as qconv2d_fused.
std::array<int64_t, 14> layer_geometry(at::IntArrayRef geometry, int64_t i, const at::Tensor& w) {
    const int64_t* g = geometry.data() + 11 * i;
    return {g[0], g[1], g[2], g[3], w.size(0), w.size(2), w.size(3), g[4], g[5], g[6], g[7], g[8], g[9], g[10]};
}

std::vector<at::Tensor> qconv2d_pack_batch(at::TensorList weights, at::IntArrayRef geometry, int64_t bits, int64_t mode,
                                           int64_t fsr, int64_t prec, at::IntArrayRef plans) {
    const int64_t n = (int64_t)weights.size();
    TORCH_CHECK((int64_t)geometry.size() == 11 * n, "po2q: pack_batch: 11 geometry ints per weight");
    TORCH_CHECK(plans.empty() || (int64_t)plans.size() == n, "po2q: pack_batch: one plan index per weight (or none)");
    if (n == 0) return {};
    check_hip_f32(weights[0], "weight");
    const DeviceGuard guard(weights[0].device());
    std::vector<PlanEntry*> es(n);
    std::vector<at::Tensor> wc(n);
    std::vector<int64_t> off(n + 1, 0);
    for (int64_t i = 0; i < n; ++i) {
        check_hip_f32(weights[i], "weight");
        TORCH_CHECK(weights[i].dim() == 4 && weights[i].device() == weights[0].device(),
                    "po2q: pack_batch: 4-D weights on one device");
        wc[i] = weights[i].contiguous();
        es[i] = plan_lookup(layer_geometry(geometry, i, wc[i]), bits, fsr, mode, prec, plans.empty() ? -1 : plans[i],
                            weights[0].device().index());
        const int pw = po2q_qconv2d_plan_packs_weight(es[i]->plan);
        TORCH_CHECK(pw >= 0, last_error());
        off[i + 1] = off[i] + (pw ? ((int64_t)es[i]->ws + 255) / 256 * 256 : 0);
    }
    at::Tensor all = at::empty({std::max<int64_t>(off[n], 256)}, weights[0].options().dtype(at::kByte));
    std::vector<at::Tensor> out(n);
    std::vector<const po2q_conv_plan*> hp;
    std::vector<const float*> wp;
    std::vector<void*> sp;
    std::vector<size_t> bp;
    for (int64_t i = 0; i < n; ++i) {
        out[i] = all.narrow(0, off[i], off[i + 1] - off[i]);
        if (off[i + 1] == off[i]) continue;
        hp.push_back(es[i]->plan);
        wp.push_back(wc[i].data_ptr<float>());
        sp.push_back(out[i].data_ptr());
        bp.push_back(es[i]->ws);
    }
    if (!hp.empty()) {
        const int st = po2q_qconv2d_plan_pack_batch((int)hp.size(), hp.data(), wp.data(), sp.data(), bp.data(),
                                                    stream_of(weights[0]));
        TORCH_CHECK(st == 0, last_error());
    }
    return out;
}

std::vector<at::Tensor> qconv2d_pack_batch_meta(at::TensorList weights, at::IntArrayRef geometry, int64_t bits,
                                                int64_t mode, int64_t fsr, int64_t prec, at::IntArrayRef plans) {
    const int64_t n = (int64_t)weights.size();
    TORCH_CHECK((int64_t)geometry.size() == 11 * n && (plans.empty() || (int64_t)plans.size() == n),
                "po2q: pack_batch: bad lists");
    std::vector<at::Tensor> out;
    for (int64_t i = 0; i < n; ++i) {
        PlanEntry* e = plan_lookup(layer_geometry(geometry, i, weights[i]), bits, fsr, mode, prec,
                                   plans.empty() ? -1 : plans[i], -1);
        const int pw = po2q_qconv2d_plan_packs_weight(e->plan);
        out.push_back(at::empty({pw > 0 ? (int64_t)e->ws : 0}, weights[i].options().dtype(at::kByte)));
    }
    return out;
}

at::Tensor qconv2d_packed(const at::Tensor& x_, const at::Tensor& w_, const at::Tensor& workspace,
                          const c10::optional<at::Tensor>& bias_, at::IntArrayRef stride, at::IntArrayRef padding,
                          at::IntArrayRef dilation, int64_t groups, int64_t bits, int64_t mode, int64_t fsr,
                          int64_t prec, int64_t plan, const c10::optional<at::Tensor>& post_scale,
                          const c10::optional<at::Tensor>& post_shift, const c10::optional<at::Tensor>& residual,
                          int64_t act) {
    if (workspace.numel() == 0)  // nothing was pre-packed: the kernel stages its own weight
        return qconv2d_impl(x_, w_, bias_, stride, padding, dilation, groups, bits, mode, fsr, prec, plan, 0,
                            post_scale, post_shift, residual, act);
    TORCH_CHECK(act >= 0 && act <= 3, "po2q: unknown activation ", act);
    const Geometry G = conv_geometry(x_, w_, bias_, stride, padding, dilation, groups);
    TORCH_CHECK(workspace.is_cuda() && workspace.scalar_type() == at::kByte && workspace.is_contiguous() &&
                    workspace.device() == x_.device(),
                "po2q: packed: the workspace must be a contiguous uint8 tensor on the input's device");
    const DeviceGuard guard(x_.device());
    PlanEntry* e = plan_lookup(G.g, bits, fsr, mode, prec, plan, x_.device().index());
    TORCH_CHECK((size_t)workspace.numel() >= e->ws,
                "po2q: packed: workspace of ", workspace.numel(), " bytes, the plan needs ", e->ws,
                " (pack it with qconv2d_pack_batch for this geometry)");
    const at::Tensor x = x_.contiguous(), w = w_.contiguous();
    c10::optional<at::Tensor> bias, ps, pb, res;
    if (bias_.has_value()) bias = bias_->contiguous();
    check_vec(post_scale, x, G.yshape[1], "post_scale");
    check_vec(post_shift, x, G.yshape[1], "post_shift");
    if (post_scale.has_value()) ps = post_scale->contiguous();
    if (post_shift.has_value()) pb = post_shift->contiguous();
    if (residual.has_value()) {
        check_hip_f32(*residual, "residual");
        TORCH_CHECK(residual->device() == x.device() && residual->sizes() == at::IntArrayRef(G.yshape),
                    "po2q: residual shape ", residual->sizes(), " does not match the output ", at::IntArrayRef(G.yshape));
        res = residual->contiguous();
    }
    at::Tensor y = at::empty(G.yshape, x.options());
    if (G.yshape[0] == 0) return y;
    const int st = po2q_qconv2d_plan_run_packed(e->plan, x.data_ptr<float>(), w.data_ptr<float>(), opt_ptr(bias),
                                                y.data_ptr<float>(), opt_ptr(ps), opt_ptr(pb), opt_ptr(res), (int)act,
                                                workspace.data_ptr(), (size_t)workspace.numel(), stream_of(x));
    TORCH_CHECK(st == 0, last_error());
    return y;
}

at::Tensor qconv2d_packed_meta(const at::Tensor& x, const at::Tensor& w, const at::Tensor&,
                               const c10::optional<at::Tensor>& bias, at::IntArrayRef stride, at::IntArrayRef padding,
                               at::IntArrayRef dilation, int64_t groups, int64_t bits, int64_t mode, int64_t fsr,
                               int64_t prec, int64_t plan, const c10::optional<at::Tensor>&,
                               const c10::optional<at::Tensor>&, const c10::optional<at::Tensor>&, int64_t) {
    return qconv2d_meta(x, w, bias, stride, padding, dilation, groups, bits, mode, fsr, prec, plan, 0);
}

// ---- one inverted-residual block (expand -> depthwise 3x3 -> project) from packed workspaces ----
// we / ws_e absent: no expand (h = x).  The workspaces come from qconv2d_pack_batch with the
// same geometry and plan indices (plans: 3 ints, or empty for -1 = tuned / heuristic).  When the
// three plans cannot run as one block (po2q_qconv2d_ir_supported) or a workspace is empty the
// three layers run one by one from their workspaces (qconv2d_packed) -- the same HIP kernels.
struct IrShape {
    int64_t N, Cin, H, W, Ch, Cout, S, Ho, Wo;
};

IrShape ir_shape(const at::Tensor& x, const c10::optional<at::Tensor>& we, const at::Tensor& wd, const at::Tensor& wp,
                 int64_t stride) {
    TORCH_CHECK(x.dim() == 4, "po2q: inverted residual: x must be 4-D [N, C, H, W]");
    TORCH_CHECK(stride == 1 || stride == 2, "po2q: inverted residual: stride must be 1 or 2");
    IrShape s{x.size(0), x.size(1), x.size(2), x.size(3), wd.size(0), wp.size(0), stride, 0, 0};
    TORCH_CHECK(wd.dim() == 4 && wd.size(1) == 1 && wd.size(2) == 3 && wd.size(3) == 3,
                "po2q: inverted residual: the depthwise weight must be [Ch, 1, 3, 3], got ", wd.sizes());
    if (we.has_value()) {
        TORCH_CHECK(we->dim() == 4 && we->size(0) == s.Ch && we->size(1) == s.Cin && we->size(2) == 1 &&
                        we->size(3) == 1,
                    "po2q: inverted residual: the expand weight must be [Ch, Cin, 1, 1] = [", s.Ch, ", ", s.Cin,
                    ", 1, 1], got ", we->sizes());
    } else {
        TORCH_CHECK(s.Cin == s.Ch, "po2q: inverted residual without expand: x has ", s.Cin,
                    " channels, the depthwise conv ", s.Ch);
    }
    TORCH_CHECK(wp.dim() == 4 && wp.size(1) == s.Ch && wp.size(2) == 1 && wp.size(3) == 1,
                "po2q: inverted residual: the project weight must be [Cout, Ch, 1, 1], got ", wp.sizes());
    s.Ho = (s.H - 1) / stride + 1;
    s.Wo = (s.W - 1) / stride + 1;
    return s;
}

at::Tensor qconv2d_ir(const at::Tensor& x_, const c10::optional<at::Tensor>& we, const at::Tensor& wd,
                      const at::Tensor& wp, const c10::optional<at::Tensor>& ws_e, const at::Tensor& ws_d,
                      const at::Tensor& ws_p, int64_t stride, int64_t bits, int64_t mode, int64_t fsr, int64_t prec,
                      const c10::optional<at::Tensor>& ps1, const c10::optional<at::Tensor>& pb1, int64_t act1,
                      const c10::optional<at::Tensor>& ps2, const c10::optional<at::Tensor>& pb2, int64_t act2,
                      const c10::optional<at::Tensor>& ps3, const c10::optional<at::Tensor>& pb3,
                      const c10::optional<at::Tensor>& residual, int64_t act3, at::IntArrayRef plans) {
    check_hip_f32(x_, "x");
    check_hip_f32(wd, "depthwise weight");
    check_hip_f32(wp, "project weight");
    if (we.has_value()) check_hip_f32(*we, "expand weight");
    const IrShape s = ir_shape(x_, we, wd, wp, stride);
    TORCH_CHECK(plans.empty() || plans.size() == 3, "po2q: inverted residual: 3 plan indices (or none)");
    TORCH_CHECK(we.has_value() == ws_e.has_value(), "po2q: inverted residual: ws_e goes with we");
    for (int64_t a : {act1, act2, act3}) TORCH_CHECK(a >= 0 && a <= 3, "po2q: unknown activation ", a);
    const int64_t pe = plans.empty() ? -1 : plans[0], pd = plans.empty() ? -1 : plans[1],
                  pp = plans.empty() ? -1 : plans[2];
    const bool have_ws = (!ws_e.has_value() || ws_e->numel() > 0) && ws_d.numel() > 0 && ws_p.numel() > 0;
    const DeviceGuard guard(x_.device());
    const int64_t dev = x_.device().index();
    PlanEntry* ee = we.has_value()
                        ? plan_lookup({s.N, s.Cin, s.H, s.W, s.Ch, 1, 1, 1, 1, 0, 0, 1, 1, 1}, bits, fsr, mode, prec, pe, dev)
                        : nullptr;
    PlanEntry* ed = plan_lookup({s.N, s.Ch, s.H, s.W, s.Ch, 3, 3, s.S, s.S, 1, 1, 1, 1, s.Ch}, bits, fsr, mode, prec,
                                pd, dev);
    PlanEntry* ep = plan_lookup({s.N, s.Ch, s.Ho, s.Wo, s.Cout, 1, 1, 1, 1, 0, 0, 1, 1, 1}, bits, fsr, mode, prec, pp,
                                dev);
    const int sup = have_ws ? po2q_qconv2d_ir_supported(ee ? ee->plan : nullptr, ed->plan, ep->plan) : 0;
    TORCH_CHECK(sup >= 0, last_error());
    if (sup == 0 || s.N == 0) {  // the layer chain from the same workspaces
        const at::Tensor empty = at::empty({0}, x_.options().dtype(at::kByte));
        at::Tensor h = x_;
        if (we.has_value())
            h = qconv2d_packed(x_, *we, ws_e->numel() ? *ws_e : empty, c10::nullopt, {1, 1}, {0, 0}, {1, 1}, 1, bits,
                               mode, fsr, prec, pe, ps1, pb1, c10::nullopt, act1);
        at::Tensor d = qconv2d_packed(h, wd, ws_d, c10::nullopt, {s.S, s.S}, {1, 1}, {1, 1}, s.Ch, bits, mode, fsr,
                                      prec, pd, ps2, pb2, c10::nullopt, act2);
        return qconv2d_packed(d, wp, ws_p, c10::nullopt, {1, 1}, {0, 0}, {1, 1}, 1, bits, mode, fsr, prec, pp, ps3,
                              pb3, residual, act3);
    }
    const at::Tensor x = x_.contiguous();
    const std::vector<int64_t> yshape{s.N, s.Cout, s.Ho, s.Wo};
    std::array<c10::optional<at::Tensor>, 6> vc;
    const c10::optional<at::Tensor>* vs[6] = {&ps1, &pb1, &ps2, &pb2, &ps3, &pb3};
    const char* names[6] = {"ps1", "pb1", "ps2", "pb2", "ps3", "pb3"};
    for (int i = 0; i < 6; ++i) {
        check_vec(*vs[i], x, i < 4 ? s.Ch : s.Cout, names[i]);
        if (vs[i]->has_value()) vc[i] = (*vs[i])->contiguous();
    }
    c10::optional<at::Tensor> res;
    if (residual.has_value()) {
        check_hip_f32(*residual, "residual");
        TORCH_CHECK(residual->device() == x.device() && residual->sizes() == at::IntArrayRef(yshape),
                    "po2q: residual shape ", residual->sizes(), " does not match the output ", at::IntArrayRef(yshape));
        res = residual->contiguous();
    }
    for (const at::Tensor* t : {&ws_d, &ws_p})
        TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kByte && t->is_contiguous() && t->device() == x.device(),
                    "po2q: inverted residual: workspaces must be contiguous uint8 tensors on the input's device");
    if (ws_e.has_value())  // NOLINT
        TORCH_CHECK(ws_e->is_cuda() && ws_e->scalar_type() == at::kByte && ws_e->is_contiguous() &&
                        ws_e->device() == x.device(),
                    "po2q: inverted residual: workspaces must be contiguous uint8 tensors on the input's device");
    at::Tensor y = at::empty(yshape, x.options());
    const int st = po2q_qconv2d_ir_f32(
        x.data_ptr<float>(), y.data_ptr<float>(), ee ? ee->plan : nullptr, ws_e.has_value() ? ws_e->data_ptr() : nullptr,
        ws_e.has_value() ? (size_t)ws_e->numel() : 0, ed->plan, ws_d.data_ptr(), (size_t)ws_d.numel(), ep->plan,
        ws_p.data_ptr(), (size_t)ws_p.numel(), opt_ptr(vc[0]), opt_ptr(vc[1]), (int)act1, opt_ptr(vc[2]),
        opt_ptr(vc[3]), (int)act2, opt_ptr(vc[4]), opt_ptr(vc[5]), opt_ptr(res), (int)act3, stream_of(x));
    TORCH_CHECK(st == 0, last_error());
    return y;
}

at::Tensor qconv2d_ir_meta(const at::Tensor& x, const c10::optional<at::Tensor>& we, const at::Tensor& wd,
                           const at::Tensor& wp, const c10::optional<at::Tensor>&, const at::Tensor&, const at::Tensor&,
                           int64_t stride, int64_t, int64_t, int64_t, int64_t, const c10::optional<at::Tensor>&,
                           const c10::optional<at::Tensor>&, int64_t, const c10::optional<at::Tensor>&,
                           const c10::optional<at::Tensor>&, int64_t, const c10::optional<at::Tensor>&,
                           const c10::optional<at::Tensor>&, const c10::optional<at::Tensor>&, int64_t,
                           at::IntArrayRef) {
    const IrShape s = ir_shape(x, we, wd, wp, stride);
    return at::empty({s.N, s.Cout, s.Ho, s.Wo}, x.options());
}

}  // namespace

TORCH_LIBRARY(po2q, m) {
    m.def("quantize(Tensor w, int bits, int mode, int fsr=1) -> Tensor");
    m.def("quantize_lin(Tensor w, int bits, int num_iters=10, int plus=0) -> Tensor");
    m.def("qconv2d(Tensor x, Tensor w, Tensor? bias, int[2] stride, int[2] padding, int[2] dilation, int groups, "
          "int bits, int mode, int fsr=1, int precision=0, int plan=-1, int autotune=0) -> Tensor");
    m.def("qconv2d_fused(Tensor x, Tensor w, Tensor? bias, int[2] stride, int[2] padding, int[2] dilation, "
          "int groups, int bits, int mode, int fsr=1, int precision=0, int plan=-1, int autotune=0, "
          "Tensor? post_scale=None, Tensor? post_shift=None, Tensor? residual=None, int act=0) -> Tensor");
    m.def("conv_wgrad(Tensor x, Tensor dy, int[] wshape, int[2] stride, int[2] padding, int[2] dilation, "
          "int groups=1) -> Tensor");
    m.def("dilate(Tensor x, int[2] stride, int[2] size) -> Tensor");
    m.def("qconv2d_pair(Tensor x, Tensor w1, Tensor w2, int bits, int mode, int fsr=1, Tensor? bias1=None, "
          "Tensor? bias2=None, Tensor? post_scale1=None, Tensor? post_shift1=None, int act1=0, "
          "Tensor? post_scale2=None, Tensor? post_shift2=None, Tensor? residual=None, int act2=0) -> Tensor");
    m.def("qconv2d_s2ds(Tensor x, Tensor w, Tensor wds, int bits, int mode, int fsr=1, Tensor? post_scale=None, "
          "Tensor? post_shift=None, int act=0, Tensor? post_scale_ds=None, Tensor? post_shift_ds=None) "
          "-> (Tensor, Tensor)");
    m.def("qconv2d_chain(Tensor x, Tensor[] weights, int bits, int mode, int fsr, Tensor?[] biases, "
          "Tensor?[] post_scales, Tensor?[] post_shifts, int[] acts=[], int[] res_from=[]) -> Tensor");
    m.def("qconv2d_pack_batch(Tensor[] weights, int[] geometry, int bits, int mode, int fsr=1, int precision=0, "
          "int[] plans=[]) -> Tensor[]");
    m.def("qconv2d_packed(Tensor x, Tensor w, Tensor workspace, Tensor? bias, int[2] stride, int[2] padding, "
          "int[2] dilation, int groups, int bits, int mode, int fsr=1, int precision=0, int plan=-1, "
          "Tensor? post_scale=None, Tensor? post_shift=None, Tensor? residual=None, int act=0) -> Tensor");
    m.def("qconv2d_ir(Tensor x, Tensor? we, Tensor wd, Tensor wp, Tensor? ws_e, Tensor ws_d, Tensor ws_p, "
          "int stride, int bits, int mode, int fsr=1, int precision=0, Tensor? ps1=None, Tensor? pb1=None, "
          "int act1=0, Tensor? ps2=None, Tensor? pb2=None, int act2=0, Tensor? ps3=None, Tensor? pb3=None, "
          "Tensor? residual=None, int act3=0, int[] plans=[]) -> Tensor");
}

TORCH_LIBRARY_IMPL(po2q, CUDA, m) {  // the HIP device (PyTorch-ROCm dispatches HIP tensors under CUDA)
    m.impl("quantize", &quantize);
    m.impl("quantize_lin", &quantize_lin);
    m.impl("qconv2d", &qconv2d);
    m.impl("qconv2d_fused", &qconv2d_fused);
    m.impl("conv_wgrad", &conv_wgrad);
    m.impl("dilate", &dilate);
    m.impl("qconv2d_pair", &qconv2d_pair);
    m.impl("qconv2d_s2ds", &qconv2d_s2ds);
    m.impl("qconv2d_chain", &qconv2d_chain);
    m.impl("qconv2d_pack_batch", &qconv2d_pack_batch);
    m.impl("qconv2d_packed", &qconv2d_packed);
    m.impl("qconv2d_ir", &qconv2d_ir);
}

TORCH_LIBRARY_IMPL(po2q, Meta, m) {
    m.impl("quantize", &same_meta);
    m.impl("quantize_lin", &same_meta);
    m.impl("qconv2d", &qconv2d_meta);
    m.impl("qconv2d_fused", &qconv2d_fused_meta);
    m.impl("conv_wgrad", &conv_wgrad_meta);
    m.impl("dilate", &dilate_meta);
    m.impl("qconv2d_pair", &qconv2d_pair_meta);
    m.impl("qconv2d_s2ds", &qconv2d_s2ds_meta);
    m.impl("qconv2d_chain", &qconv2d_chain_meta);
    m.impl("qconv2d_pack_batch", &qconv2d_pack_batch_meta);
    m.impl("qconv2d_packed", &qconv2d_packed_meta);
    m.impl("qconv2d_ir", &qconv2d_ir_meta);
}
