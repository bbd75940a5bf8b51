// C ABI of the po2q library (include/po2q.h): argument validation, workspace
// layout and dispatch.  Everything is enqueued on the caller's stream; nothing
// here allocates device memory or synchronises.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <algorithm>
#include <new>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/po2q.h"
#include "po2q_epi.h"
#include "po2q_internal.h"

namespace po2q {
static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
}  // namespace po2q

using namespace po2q;

namespace {

constexpr size_t kAlign = 256;
size_t align_up(size_t v) { return (v + kAlign - 1) / kAlign * kAlign; }

bool check_mode_bits(int mode, int bits, bool allow_none) {
    if (mode != PO2Q_MODE_PO2 && mode != PO2Q_MODE_PO2_PLUS && !(allow_none && mode == PO2Q_MODE_NONE)) {
        set_error("po2q: unknown quantizer mode " + std::to_string(mode));
        return false;
    }
    if (mode != PO2Q_MODE_NONE && (bits < 1 || bits > 16)) {
        set_error("po2q: bits must be in [1, 16], got " + std::to_string(bits));
        return false;
    }
    return true;
}

int hip_status(hipError_t e, const char* what) {
    if (e == hipSuccess) return PO2Q_OK;
    set_error(std::string("po2q: ") + what + ": " + hipGetErrorString(e));
    return PO2Q_ERR_HIP;
}

}  // namespace

extern "C" {

const char* po2q_version(void) { return "po2q 0.1.0 (gfx950)"; }

const char* po2q_last_error(void) { return g_last_error.c_str(); }

size_t po2q_quantize_workspace_bytes(int64_t n) {
    if (n <= 0) return 0;
    return align_up((size_t)absmax_blocks(n) * sizeof(uint64_t));  // fp64 partials are 8 bytes
}

int po2q_quantize_f32(const float* w, float* out, int64_t n, int bits, int fsr, int mode, void* workspace,
                      size_t workspace_bytes, void* stream) {
    if (n <= 0) {
        set_error("po2q: max(): Expected reduction dim to be specified for input.numel() == 0");
        return PO2Q_ERR_INVALID;
    }
    if (!check_mode_bits(mode, bits, false)) return PO2Q_ERR_INVALID;
    if (!w || !out || !workspace) {
        set_error("po2q: null pointer");
        return PO2Q_ERR_INVALID;
    }
    if (workspace_bytes < po2q_quantize_workspace_bytes(n)) {
        set_error("po2q: quantize workspace too small");
        return PO2Q_ERR_WORKSPACE;
    }
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    unsigned* partial = reinterpret_cast<unsigned*>(workspace);
    const int nb = absmax_blocks(n);
    int st = hip_status(launch_absmax(w, n, partial, nb, s), "absmax launch");
    if (st) return st;
    return hip_status(launch_quantize_plain(w, n, partial, nb, bits, fsr, mode, out, s), "quantize launch");
}

}  // extern "C"

// fp64 / bf16 weights (the reference keeps the dtype, quantizers.py:19-56)
template <typename T>
static int quantize_dt(const T* w, T* out, int64_t n, int bits, int fsr, int mode, void* workspace,
                       size_t workspace_bytes, void* stream) {
    if (n <= 0) {
        set_error("po2q: max(): Expected reduction dim to be specified for input.numel() == 0");
        return PO2Q_ERR_INVALID;
    }
    if (!check_mode_bits(mode, bits, false)) return PO2Q_ERR_INVALID;
    if (!w || !out || !workspace) {
        set_error("po2q: null pointer");
        return PO2Q_ERR_INVALID;
    }
    if (workspace_bytes < po2q_quantize_workspace_bytes(n)) {
        set_error("po2q: quantize workspace too small");
        return PO2Q_ERR_WORKSPACE;
    }
    return hip_status(launch_quantize_dt<T>(w, out, n, bits, fsr, mode, reinterpret_cast<uint64_t*>(workspace),
                                            absmax_blocks(n), reinterpret_cast<hipStream_t>(stream)),
                      "quantize launch");
}

extern "C" {

int po2q_quantize_f64(const double* w, double* out, int64_t n, int bits, int fsr, int mode, void* workspace,
                      size_t workspace_bytes, void* stream) {
    return quantize_dt<double>(w, out, n, bits, fsr, mode, workspace, workspace_bytes, stream);
}

int po2q_quantize_bf16(const uint16_t* w, uint16_t* out, int64_t n, int bits, int fsr, int mode, void* workspace,
                       size_t workspace_bytes, void* stream) {
    return quantize_dt<uint16_t>(w, out, n, bits, fsr, mode, workspace, workspace_bytes, stream);
}

int po2q_quantize_lin_f32(const float* w, float* out, int64_t d0, int64_t d1, int64_t d2, int64_t d3, int bits,
                          int num_iters, int plus, void* stream) {
    if (d0 <= 0 || d1 <= 0 || d2 <= 0 || d3 <= 0) {
        set_error("po2q: max(): Expected reduction dim to have non-zero size (lin quantizer needs a non-empty "
                  "4-D weight)");
        return PO2Q_ERR_INVALID;
    }
    if (bits < 1 || bits > 16 || num_iters < 0 || (plus != 0 && plus != 1)) {
        set_error("po2q: lin quantizer needs 1 <= bits <= 16, num_iters >= 0, plus in {0, 1}");
        return PO2Q_ERR_INVALID;
    }
    if ((int64_t)d0 * d2 * d3 > (1LL << 30) || d1 > (1LL << 30) || d0 * d1 * d2 * d3 > (1LL << 40)) {
        set_error("po2q: lin quantizer weight too large");
        return PO2Q_ERR_INVALID;
    }
    if (!w || !out) {
        set_error("po2q: null pointer");
        return PO2Q_ERR_INVALID;
    }
    return hip_status(launch_quantize_lin(w, out, (int)d0, (int)d1, (int)(d2 * d3), bits, num_iters, plus,
                                          reinterpret_cast<hipStream_t>(stream)),
                      "lin quantize launch");
}

// Workspace layout: [absmax partials][scale (bf16x3)][packed weights]
struct WsLayout {
    size_t part_bytes, scale_off, packed_off, total;
    int nparts;  // 0: absmax fused into the bf16x3 pack kernel
};

static WsLayout ws_layout(const ConvPlan& p, int mode) {
    WsLayout L;
    const int64_t nw = (int64_t)p.K * p.Cg * p.R * p.S;
    const bool fused = (is_bf16x3_kind(p.kind) || p.kind == KIND_DEPTHWISE) &&
                       nw <= kFusedAbsmaxMax;
    L.nparts = (mode == PO2Q_MODE_NONE || fused) ? 0 : absmax_blocks(nw);
    L.part_bytes = align_up((size_t)absmax_blocks(nw) * sizeof(unsigned));
    L.scale_off = L.part_bytes;
    L.packed_off = L.scale_off + kAlign;
    L.total = L.packed_off + align_up((size_t)p.packed_floats * sizeof(float));
    return L;
}

size_t po2q_qconv2d_workspace_bytes(int64_t N, int64_t C, int64_t H, int64_t W, int64_t K, int64_t R,
                                       int64_t S, int64_t stride_h, int64_t stride_w, int64_t pad_h, int64_t pad_w,
                                       int64_t dil_h, int64_t dil_w, int64_t groups, int bits, int fsr, int mode,
                                       int flags) {
    // the maximum over every plan the autotuner may pick, so one workspace serves
    // the heuristic plan, the autotune sweep and the tuned plan alike
    std::vector<ConvPlan> cands;
    if (!plan_candidates(cands, N, C, H, W, K, R, S, stride_h, stride_w, pad_h, pad_w, dil_h, dil_w, groups, mode,
                         bits, fsr, flags))
        return 0;
    ConvPlan p;
    if (!make_plan(p, N, C, H, W, K, R, S, stride_h, stride_w, pad_h, pad_w, dil_h, dil_w, groups, mode, bits, fsr,
                   flags))
        return 0;
    size_t total = ws_layout(p, mode).total;
    for (const ConvPlan& c : cands) total = std::max(total, ws_layout(c, mode).total);
    return total;
}

static int check_conv_args(const float* x, const float* w, float* y, void* workspace, int mode, int bits,
                           int flags) {
    if (!check_mode_bits(mode, bits, true)) return PO2Q_ERR_INVALID;
    if (flags < PO2Q_PREC_AUTO || flags > PO2Q_PREC_BF16X3) {
        set_error("po2q: unknown precision flag " + std::to_string(flags));
        return PO2Q_ERR_INVALID;
    }
    if (!x || !w || !y || !workspace) {
        set_error("po2q: null pointer");
        return PO2Q_ERR_INVALID;
    }
    return PO2Q_OK;
}

static inline void clamp_window_host(int bits, int fsr, int& lo, int& hi) {
    lo = fsr - (1 << (bits - 1));
    hi = fsr - 1;
}

// Whether run_plan's RUN_PACK phase enqueues anything for plan p: not for the plans that
// stage their weight in-kernel (bf16x3 with fused staging) or read it as given (fp32 stems /
// pointwise of mode none).
static bool plan_packs_weight(const ConvPlan& p, int /*mode*/) {
    if (p.kind == KIND_DIRECT_F32 || p.kind == KIND_PW_F32) return false;
    if (is_bf16x3_kind(p.kind) && p.fp) return false;
    return true;
}

// phases of run_plan: the weight quantize + pack into the workspace, the conv from it
enum { RUN_PACK = 1, RUN_CONV = 2, RUN_ALL = 3 };

// Enqueue the fused quantize(+pack) and conv of plan p on stream s (+ the epilogue e:
// in the row kernels' store epilogue where they support it, else one elementwise pass).
static int run_plan(const ConvPlan& p, const float* x, const float* w, const float* bias, float* y, int bits, int fsr,
                    int mode, void* workspace, size_t workspace_bytes, hipStream_t s,
                    const ConvEpi& e = ConvEpi{nullptr, nullptr, nullptr, 0}, int phases = RUN_ALL) {
    const WsLayout L = ws_layout(p, mode);
    if (workspace_bytes < L.total) {
        set_error("po2q: conv workspace too small (need " + std::to_string(L.total) + " bytes)");
        return PO2Q_ERR_WORKSPACE;
    }
    char* ws = reinterpret_cast<char*>(workspace);
    unsigned* partial = reinterpret_cast<unsigned*>(ws);
    float* scale = reinterpret_cast<float*>(ws + L.scale_off);
    void* packed = ws + L.packed_off;
    const int64_t nw = (int64_t)p.K * p.Cg * p.R * p.S;
    int st;
    if (p.kind == KIND_DIRECT_F32 || p.kind == KIND_PW_F32) {  // mode none: the weight as given, no pack
        if (!(phases & RUN_CONV)) return PO2Q_OK;
        if (!w) {
            set_error("po2q: this fp32 plan reads the weight as given: it needs w (no packed form)");
            return PO2Q_ERR_INVALID;
        }
        return hip_status(launch_conv_f32s(p, x, w, bias, y, e.ps, e.pb, e.res, e.act, s), "conv launch");
    }
    if ((phases & RUN_PACK) && L.nparts > 0) {
        st = hip_status(launch_absmax(w, nw, partial, L.nparts, s), "absmax launch");
        if (st) return st;
    }
    if (is_bf16x3_kind(p.kind)) {
        // fused weight staging (row plans with fp): the conv quantizes + packs the weight
        // itself -- one launch, nothing in the workspace
        WQuant q;
        if (p.fp) {
            int lo, hi;
            clamp_window_host(bits, fsr, lo, hi);
            q.w = w;
            q.n = (int)nw;
            q.lo = lo;
            q.hi = hi;
            q.mode = mode - 1;
        }
        if ((phases & RUN_PACK) && !p.fp) {
            st = hip_status(launch_pack_bf16x3(p, w, partial, L.nparts, bits, fsr, mode,
                                               reinterpret_cast<uint16_t*>(packed), scale, s),
                            "weight pack launch");
            if (st) return st;
        }
        if (!(phases & RUN_CONV)) return PO2Q_OK;
        const uint16_t* pk = reinterpret_cast<const uint16_t*>(packed);
        if (p.kind == KIND_BF16X3_PW)  // affine, residual and activation all in the kernel's stores
            return hip_status(launch_conv_pw(p, x, pk, scale, bias, y, e.ps, e.pb, e.res, e.act, s), "conv launch");
        if (p.kind == KIND_BF16X3_IMG)  // the same
            return hip_status(launch_conv_img(p, x, pk, scale, bias, y, e.ps, e.pb, e.res, e.act, s), "conv launch");
        hipError_t he;
        bool fused_affine = false;
        if (p.kind == KIND_BF16X3_DMA) {
            he = launch_conv_bf16x3_dma(p, x, pk, scale, bias, y, s);
        } else if (p.kind == KIND_BF16X3_ROWS && e.res && rows_res_ok(p)) {
            // affine, residual and activation all in the kernel's stores
            st = hip_status(launch_conv_rows_res(p, x, pk, scale, bias, y, e.ps, e.pb, e.res, e.act, s, q),
                            "conv launch");
            return st;
        } else if (p.kind == KIND_BF16X3_ROWS && e.any()) {
            // affine (+ activation unless a residual must be added first) in the kernel
            he = launch_conv_bf16x3_rows_epi(p, x, pk, scale, bias, y, e.ps, e.pb, e.res ? 0 : e.act, s, q);
            fused_affine = true;
        } else if (p.kind == KIND_BF16X3_ROWS) {
            he = launch_conv_bf16x3_rows(p, x, pk, scale, bias, y, s, q);
        } else {
            he = launch_conv_bf16x3(p, x, pk, scale, bias, y, s);
        }
        st = hip_status(he, "conv launch");
        if (st || !e.any() || (fused_affine && !e.res)) return st;
        return hip_status(launch_epilogue(y, p.N, p.K, (int64_t)p.P * p.Q, e, fused_affine, s), "epilogue launch");
    }
    if (phases & RUN_PACK) {
        st = hip_status(
            launch_pack_weights(p, w, partial, L.nparts, bits, fsr, mode, reinterpret_cast<float*>(packed), s),
            "weight pack launch");
        if (st) return st;
    }
    if (!(phases & RUN_CONV)) return PO2Q_OK;
    if (dw3_plan_ok(p))  // depthwise LDS-halo kernel: the whole epilogue in its stores
        return hip_status(launch_conv_dw3(p, x, reinterpret_cast<const float*>(packed), bias, y, e.ps, e.pb, e.res,
                                          e.act, s),
                          "conv launch");
    if (p.kind == KIND_DEPTHWISE && e.any())  // one-output-per-lane depthwise: the epilogue in its store too
        return hip_status(launch_conv_depthwise_epi(p, x, reinterpret_cast<const float*>(packed), bias, y, e.ps, e.pb,
                                                    e.res, e.act, s),
                          "conv launch");
    st = hip_status(launch_conv(p, x, reinterpret_cast<const float*>(packed), bias, y, s), "conv launch");
    if (st || !e.any()) return st;
    return hip_status(launch_epilogue(y, p.N, p.K, (int64_t)p.P * p.Q, e, false, s), "epilogue launch");
}

// Whether run_plan needs its own elementwise pass over y for an eval epilogue (BN affine + activation,
// no residual): the plans whose conv kernel cannot apply it in its stores.
static bool plan_needs_epilogue_pass(const ConvPlan& p) {
    if (p.kind == KIND_BF16X3_PW || p.kind == KIND_BF16X3_IMG || p.kind == KIND_BF16X3_ROWS) return false;
    if (p.kind == KIND_DIRECT_F32 || p.kind == KIND_PW_F32 || p.kind == KIND_DEPTHWISE) return false;
    return true;  // bf16x3 tile / DMA kernels, the fp32 MFMA kernel
}

static const char* kKindNames[] = {"mfma_f32", "depthwise", "bf16x3", "bf16x3_dma", "bf16x3_rows", "bf16x3_pw",
                                   "direct_f32", "pw_f32", "bf16x3_img"};

static void describe_plan(const ConvPlan& p, char* buf, size_t len) {
    snprintf(buf, len,
             "kind=%s CC=%d NT=%d MI=%d NJ=%d vr=%d tile=%dx%d tiles=%dx%d halo=%dx%d chunks=%d kblocks=%d ksteps=%d "
             "lds=%zu blocks=%lld waves=%d ov=%d wstream=%d pd=%d nts=%d var=%d fp=%d",
             kKindNames[p.kind], p.CC, p.NT, p.MI, p.NJ, p.vrx, p.TP, p.TQ, p.tilesP, p.tilesQ, p.HH, p.WW,
             p.nchunks, p.kblocks, p.steps, p.lds_bytes, (long long)p.blocks,
             p.kind == KIND_BF16X3_DMA ? p.dma_waves : 4, p.dma_ov,
             p.kind == KIND_BF16X3_DMA ? (p.dma_nw > 0) : (p.nchunks > 1 || p.kblocks > 1),
             (p.kind == KIND_BF16X3 || p.kind == KIND_BF16X3_ROWS) ? p.pd : 0, p.nts,
             p.kind == KIND_BF16X3_ROWS ? p.PS : 0, p.fp);
}

int po2q_qconv2d_f32(const float* x, const float* w, const float* bias, float* y, int64_t N, int64_t C, int64_t H,
                     int64_t W, int64_t K, int64_t R, int64_t S, int64_t stride_h, int64_t stride_w, int64_t pad_h,
                     int64_t pad_w, int64_t dil_h, int64_t dil_w, int64_t groups, int bits, int fsr, int mode,
                     int flags, void* workspace, size_t workspace_bytes, void* stream) {
    int st = check_conv_args(x, w, y, workspace, mode, bits, flags);
    if (st) return st;
    ConvPlan p;
    if (!make_plan(p, N, C, H, W, K, R, S, stride_h, stride_w, pad_h, pad_w, dil_h, dil_w, groups, mode, bits, fsr,
                   flags))
        return flags == PO2Q_PREC_BF16X3 ? PO2Q_ERR_UNSUPPORTED : PO2Q_ERR_INVALID;
    return run_plan(p, x, w, bias, y, bits, fsr, mode, workspace, workspace_bytes,
                    reinterpret_cast<hipStream_t>(stream));
}

int po2q_qconv2d_fused_f32(const float* x, const float* w, const float* bias, float* y, int64_t N, int64_t C,
                           int64_t H, int64_t W, int64_t K, int64_t R, int64_t S, int64_t stride_h, int64_t stride_w,
                           int64_t pad_h, int64_t pad_w, int64_t dil_h, int64_t dil_w, int64_t groups, int bits,
                           int fsr, int mode, int flags, const float* post_scale, const float* post_shift,
                           const float* residual, int act, void* workspace, size_t workspace_bytes, void* stream) {
    int st = check_conv_args(x, w, y, workspace, mode, bits, flags);
    if (st) return st;
    if (act < PO2Q_ACT_NONE || act > PO2Q_ACT_SILU) {
        set_error("po2q: unknown activation " + std::to_string(act));
        return PO2Q_ERR_INVALID;
    }
    ConvPlan p;
    if (!make_plan(p, N, C, H, W, K, R, S, stride_h, stride_w, pad_h, pad_w, dil_h, dil_w, groups, mode, bits, fsr,
                   flags))
        return flags == PO2Q_PREC_BF16X3 ? PO2Q_ERR_UNSUPPORTED : PO2Q_ERR_INVALID;
    const ConvEpi e{post_scale, post_shift, residual, act};
    return run_plan(p, x, w, bias, y, bits, fsr, mode, workspace, workspace_bytes,
                    reinterpret_cast<hipStream_t>(stream), e);
}

int po2q_qconv2d_autotune(const float* x, const float* w, const float* bias, float* y, int64_t N, int64_t C,
                          int64_t H, int64_t W, int64_t K, int64_t R, int64_t S, int64_t stride_h, int64_t stride_w,
                          int64_t pad_h, int64_t pad_w, int64_t dil_h, int64_t dil_w, int64_t groups, int bits,
                          int fsr, int mode, int flags, void* workspace, size_t workspace_bytes, void* stream,
                          char* buf, size_t len) {
    int st = check_conv_args(x, w, y, workspace, mode, bits, flags);
    if (st) return st;
    std::vector<ConvPlan> cands;
    if (!plan_candidates(cands, N, C, H, W, K, R, S, stride_h, stride_w, pad_h, pad_w, dil_h, dil_w, groups, mode,
                         bits, fsr, flags))
        return flags == PO2Q_PREC_BF16X3 ? PO2Q_ERR_UNSUPPORTED : PO2Q_ERR_INVALID;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    st = hip_status(hipStreamIsCapturing(s, &cs), "stream capture query");
    if (st) return st;
    if (cs != hipStreamCaptureStatusNone) {
        set_error("po2q: autotune synchronises the stream; run it before graph capture");
        return PO2Q_ERR_INVALID;
    }
    hipEvent_t e0, e1;
    st = hip_status(hipEventCreate(&e0), "event create");
    if (st) return st;
    if ((st = hip_status(hipEventCreate(&e1), "event create"))) {
        (void)hipEventDestroy(e0);
        return st;
    }
    // Two passes over the candidates, each run timed on its own and the minimum kept:
    // the first candidates of a cold GPU run at ramping clocks, so a single pass
    // would favour late candidates.
    constexpr int kPasses = 2, kReps = 2;
    int best = -1;
    std::vector<float> tmin(cands.size(), 1e30f);
    for (int pass = 0; pass < kPasses && !st; ++pass) {
        for (int i = 0; i < (int)cands.size() && !st; ++i) {
            st = run_plan(cands[i], x, w, bias, y, bits, fsr, mode, workspace, workspace_bytes, s);  // untimed
            for (int r = 0; r < kReps && !st; ++r) {
                st = hip_status(hipEventRecord(e0, s), "event record");
                if (!st) st = run_plan(cands[i], x, w, bias, y, bits, fsr, mode, workspace, workspace_bytes, s);
                if (!st) st = hip_status(hipEventRecord(e1, s), "event record");
                if (!st) st = hip_status(hipEventSynchronize(e1), "autotune run");
                float ms = 0.f;
                if (!st) st = hip_status(hipEventElapsedTime(&ms, e0, e1), "event time");
                if (!st) tmin[i] = std::min(tmin[i], ms);
            }
        }
    }
    // The model forwards call almost every conv with the eval BatchNorm (+ activation) after it
    // (QuantizedConv2d.fused): a plan that cannot apply it in its stores pays one more pass over y.
    // Charge that pass (timed once here: read + write of y) to those plans, so e.g. an unquantized
    // stem takes the direct kernel with its fused epilogue over an fp32 MFMA plan that is faster
    // alone but needs the pack, the conv and the pass (31 vs ~10 us, MobileNetV2 @32).
    float epi_ms = 0.f;
    if (!st) {
        bool any = false;
        for (const ConvPlan& c : cands) any = any || plan_needs_epilogue_pass(c);
        const ConvEpi ep{nullptr, nullptr, nullptr, PO2Q_ACT_RELU};
        for (int r = 0; any && r < 3 && !st; ++r) {
            st = hip_status(hipEventRecord(e0, s), "event record");
            if (!st) st = hip_status(launch_epilogue(y, N, K, (int64_t)cands[0].P * cands[0].Q, ep, false, s), "epilogue");
            if (!st) st = hip_status(hipEventRecord(e1, s), "event record");
            if (!st) st = hip_status(hipEventSynchronize(e1), "autotune run");
            float ms = 0.f;
            if (!st) st = hip_status(hipEventElapsedTime(&ms, e0, e1), "event time");
            if (!st && r > 0) epi_ms = r == 1 ? ms : std::min(epi_ms, ms);
        }
    }
    for (int i = 0; i < (int)cands.size(); ++i)
        if (plan_needs_epilogue_pass(cands[i])) tmin[i] += epi_ms;
    for (int i = 0; i < (int)cands.size(); ++i)
        if (best < 0 || tmin[i] < tmin[best]) best = i;
    // within 1 % (timing noise), prefer a plan with fused weight staging: one launch per
    // layer instead of pack + conv (fewer kernel boundaries in a real chain)
    if (best >= 0 && !cands[best].fp) {
        int bf = -1;
        for (int i = 0; i < (int)cands.size(); ++i)
            if (cands[i].fp && tmin[i] <= 1.01f * tmin[best] && (bf < 0 || tmin[i] < tmin[bf])) bf = i;
        if (bf >= 0) best = bf;
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (st) return st;
    tuned_store(cands[best], mode, bits, fsr, flags);
    if (buf && len) describe_plan(cands[best], buf, len);
    // leave y holding the chosen plan's output
    return run_plan(cands[best], x, w, bias, y, bits, fsr, mode, workspace, workspace_bytes, s);
}

int po2q_qconv2d_plans(int64_t N, int64_t C, int64_t H, int64_t W, int64_t K, int64_t R, int64_t S,
                       int64_t stride_h, int64_t stride_w, int64_t pad_h, int64_t pad_w, int64_t dil_h,
                       int64_t dil_w, int64_t groups, int bits, int fsr, int mode, int flags, int index, char* buf,
                       size_t len) {
    std::vector<ConvPlan> cands;
    if (!plan_candidates(cands, N, C, H, W, K, R, S, stride_h, stride_w, pad_h, pad_w, dil_h, dil_w, groups, mode,
                         bits, fsr, flags))
        return -(flags == PO2Q_PREC_BF16X3 ? PO2Q_ERR_UNSUPPORTED : PO2Q_ERR_INVALID);
    if (buf && len && index >= 0 && index < (int)cands.size()) describe_plan(cands[index], buf, len);
    return (int)cands.size();
}

int po2q_qconv2d_f32_plan(int index, const float* x, const float* w, const float* bias, float* y, int64_t N,
                          int64_t C, int64_t H, int64_t W, int64_t K, int64_t R, int64_t S, int64_t stride_h,
                          int64_t stride_w, int64_t pad_h, int64_t pad_w, int64_t dil_h, int64_t dil_w,
                          int64_t groups, int bits, int fsr, int mode, int flags, void* workspace,
                          size_t workspace_bytes, void* stream) {
    int st = check_conv_args(x, w, y, workspace, mode, bits, flags);
    if (st) return st;
    std::vector<ConvPlan> cands;
    if (!plan_candidates(cands, N, C, H, W, K, R, S, stride_h, stride_w, pad_h, pad_w, dil_h, dil_w, groups, mode,
                         bits, fsr, flags))
        return flags == PO2Q_PREC_BF16X3 ? PO2Q_ERR_UNSUPPORTED : PO2Q_ERR_INVALID;
    if (index < 0 || index >= (int)cands.size()) {
        set_error("po2q: plan index " + std::to_string(index) + " out of range [0, " +
                  std::to_string(cands.size()) + ")");
        return PO2Q_ERR_INVALID;
    }
    return run_plan(cands[index], x, w, bias, y, bits, fsr, mode, workspace, workspace_bytes,
                    reinterpret_cast<hipStream_t>(stream));
}

// Plan `index` (>= 0: a candidate of plan_candidates, -1: the tuned / heuristic plan).
static int pick_plan(ConvPlan& p, int index, int64_t N, int64_t C, int64_t H, int64_t W, int64_t K, int64_t R,
                     int64_t S, int64_t sh, int64_t sw, int64_t ph, int64_t pw, int64_t dh, int64_t dw,
                     int64_t groups, int mode, int bits, int fsr, int flags) {
    if (index < 0) {
        if (!make_plan(p, N, C, H, W, K, R, S, sh, sw, ph, pw, dh, dw, groups, mode, bits, fsr, flags))
            return flags == PO2Q_PREC_BF16X3 ? PO2Q_ERR_UNSUPPORTED : PO2Q_ERR_INVALID;
        return PO2Q_OK;
    }
    std::vector<ConvPlan> cands;
    if (!plan_candidates(cands, N, C, H, W, K, R, S, sh, sw, ph, pw, dh, dw, groups, mode, bits, fsr, flags))
        return flags == PO2Q_PREC_BF16X3 ? PO2Q_ERR_UNSUPPORTED : PO2Q_ERR_INVALID;
    if (index >= (int)cands.size()) {
        set_error("po2q: plan index " + std::to_string(index) + " out of range [0, " + std::to_string(cands.size()) +
                  ")");
        return PO2Q_ERR_INVALID;
    }
    p = cands[index];
    return PO2Q_OK;
}

// The two-enqueue form stages the weight in the workspace: a plan with fused weight
// staging (fp) runs as its pre-packed twin (same kernel otherwise, also a candidate).
static int pick_split_plan(ConvPlan& p, int index, int64_t N, int64_t C, int64_t H, int64_t W, int64_t K, int64_t R,
                           int64_t S, int64_t sh, int64_t sw, int64_t ph, int64_t pw, int64_t dh, int64_t dw,
                           int64_t groups, int mode, int bits, int fsr, int flags) {
    const int st = pick_plan(p, index, N, C, H, W, K, R, S, sh, sw, ph, pw, dh, dw, groups, mode, bits, fsr, flags);
    if (st) return st;
    // plans with no packed form: the stride-2 full-row kernel only exists with fused staging,
    // and the unquantized fp32 kernels (direct stem, pointwise) read the weight as given and
    // pack nothing, so a split enqueue would run them without a weight.  Take the first
    // candidate that reads a packed weight instead (for mode none: the fp32 MFMA kernel).
    auto unpacked = [](const ConvPlan& c) {
        return (c.kind == KIND_BF16X3_ROWS && c.vrx == 5) || c.kind == KIND_DIRECT_F32 || c.kind == KIND_PW_F32;
    };
    if (unpacked(p)) {
        std::vector<ConvPlan> cands;
        if (!plan_candidates(cands, N, C, H, W, K, R, S, sh, sw, ph, pw, dh, dw, groups, mode, bits, fsr, flags))
            return PO2Q_ERR_INVALID;
        bool found = false;
        for (const ConvPlan& c : cands)
            if (!c.fp && !unpacked(c)) {
                p = c;
                found = true;
                break;
            }
        if (!found) {
            set_error("po2q: no pre-packed plan for this shape (split enqueue)");
            return PO2Q_ERR_UNSUPPORTED;
        }
    }
    p.fp = 0;
    return PO2Q_OK;
}

int po2q_qconv2d_pack_f32(int plan, const float* w, int64_t N, int64_t C, int64_t H, int64_t W, int64_t K,
                          int64_t R, int64_t S, int64_t stride_h, int64_t stride_w, int64_t pad_h, int64_t pad_w,
                          int64_t dil_h, int64_t dil_w, int64_t groups, int bits, int fsr, int mode, int flags,
                          void* workspace, size_t workspace_bytes, void* stream) {
    // the conv-argument checks of po2q_qconv2d_f32 (x and y are not touched here)
    int st = check_conv_args(w, w, const_cast<float*>(w), workspace, mode, bits, flags);
    if (st) return st;
    ConvPlan p;
    st = pick_split_plan(p, plan, N, C, H, W, K, R, S, stride_h, stride_w, pad_h, pad_w, dil_h, dil_w, groups, mode,
                         bits, fsr, flags);
    if (st) return st;
    return run_plan(p, nullptr, w, nullptr, nullptr, bits, fsr, mode, workspace, workspace_bytes,
                    reinterpret_cast<hipStream_t>(stream), ConvEpi{nullptr, nullptr, nullptr, 0}, RUN_PACK);
}

int po2q_qconv2d_packed_f32(int plan, const float* x, const float* bias, float* y, int64_t N, int64_t C, int64_t H,
                            int64_t W, int64_t K, int64_t R, int64_t S, int64_t stride_h, int64_t stride_w,
                            int64_t pad_h, int64_t pad_w, int64_t dil_h, int64_t dil_w, int64_t groups, int bits,
                            int fsr, int mode, int flags, const void* workspace, size_t workspace_bytes,
                            void* stream) {
    int st = check_conv_args(x, x, y, const_cast<void*>(workspace), mode, bits, flags);
    if (st) return st;
    ConvPlan p;
    st = pick_split_plan(p, plan, N, C, H, W, K, R, S, stride_h, stride_w, pad_h, pad_w, dil_h, dil_w, groups, mode,
                         bits, fsr, flags);
    if (st) return st;
    return run_plan(p, x, nullptr, bias, y, bits, fsr, mode, const_cast<void*>(workspace), workspace_bytes,
                    reinterpret_cast<hipStream_t>(stream), ConvEpi{nullptr, nullptr, nullptr, 0}, RUN_CONV);
}

int po2q_qconv2d_describe(int64_t N, int64_t C, int64_t H, int64_t W, int64_t K, int64_t R, int64_t S,
                          int64_t stride_h, int64_t stride_w, int64_t pad_h, int64_t pad_w, int64_t dil_h,
                          int64_t dil_w, int64_t groups, int bits, int fsr, int mode, int flags, char* buf,
                          size_t len) {
    ConvPlan p;
    if (!buf || len == 0) {
        set_error("po2q: describe needs a buffer");
        return PO2Q_ERR_INVALID;
    }
    if (!make_plan(p, N, C, H, W, K, R, S, stride_h, stride_w, pad_h, pad_w, dil_h, dil_w, groups, mode, bits, fsr,
                   flags))
        return PO2Q_ERR_INVALID;
    describe_plan(p, buf, len);
    return PO2Q_OK;
}

}  // extern "C"

// ------------------------------------------------------------------ plan handles --
struct po2q_conv_plan {
    po2q::ConvPlan p;
    int bits, fsr, mode;
    size_t ws;
};

int po2q_qconv2d_plan_create(po2q_conv_plan** out, int index, int64_t N, int64_t C, int64_t H, int64_t W, int64_t K,
                             int64_t R, int64_t S, int64_t stride_h, int64_t stride_w, int64_t pad_h, int64_t pad_w,
                             int64_t dil_h, int64_t dil_w, int64_t groups, int bits, int fsr, int mode, int flags) {
    using namespace po2q;
    if (!out) {
        set_error("po2q: null plan output pointer");
        return PO2Q_ERR_INVALID;
    }
    *out = nullptr;
    if (!check_mode_bits(mode, bits, true)) return PO2Q_ERR_INVALID;
    if (flags < PO2Q_PREC_AUTO || flags > PO2Q_PREC_BF16X3) {
        set_error("po2q: unknown precision flag " + std::to_string(flags));
        return PO2Q_ERR_INVALID;
    }
    ConvPlan p;
    const int st = pick_plan(p, index, N, C, H, W, K, R, S, stride_h, stride_w, pad_h, pad_w, dil_h, dil_w, groups,
                             mode, bits, fsr, flags);
    if (st) return st;
    po2q_conv_plan* h = new (std::nothrow) po2q_conv_plan;
    if (!h) {
        set_error("po2q: out of host memory");
        return PO2Q_ERR_INVALID;
    }
    h->p = p;
    h->bits = bits;
    h->fsr = fsr;
    h->mode = mode;
    h->ws = std::max<size_t>(ws_layout(p, mode).total, 256);
    *out = h;
    return PO2Q_OK;
}

size_t po2q_qconv2d_plan_workspace_bytes(const po2q_conv_plan* plan) { return plan ? plan->ws : 0; }

int po2q_qconv2d_plan_run(const po2q_conv_plan* plan, const float* x, const float* w, const float* bias, float* y,
                          const float* post_scale, const float* post_shift, const float* residual, int act,
                          void* workspace, size_t workspace_bytes, void* stream) {
    using namespace po2q;
    if (!plan) {
        set_error("po2q: null plan");
        return PO2Q_ERR_INVALID;
    }
    if (!x || !w || !y || !workspace) {
        set_error("po2q: null pointer");
        return PO2Q_ERR_INVALID;
    }
    if (act < PO2Q_ACT_NONE || act > PO2Q_ACT_SILU) {
        set_error("po2q: unknown activation " + std::to_string(act));
        return PO2Q_ERR_INVALID;
    }
    const ConvEpi e{post_scale, post_shift, residual, act};
    return run_plan(plan->p, x, w, bias, y, plan->bits, plan->fsr, plan->mode, workspace, workspace_bytes,
                    reinterpret_cast<hipStream_t>(stream), e);
}

int po2q_qconv2d_plan_pack_batch(int n, const po2q_conv_plan* const* plans, const float* const* w,
                                 void* const* workspace, const size_t* workspace_bytes, void* stream) {
    using namespace po2q;
    if (n < 0 || (n > 0 && (!plans || !w || !workspace || !workspace_bytes))) {
        set_error("po2q: pack batch: null arrays");
        return PO2Q_ERR_INVALID;
    }
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    std::vector<PackReq> reqs;
    for (int i = 0; i < n; ++i) {
        const po2q_conv_plan* h = plans[i];
        if (!h || !w[i] || !workspace[i]) {
            set_error("po2q: pack batch: null plan, weight or workspace");
            return PO2Q_ERR_INVALID;
        }
        const ConvPlan& p = h->p;
        const WsLayout L = ws_layout(p, h->mode);
        if (workspace_bytes[i] < L.total) {
            set_error("po2q: pack batch: workspace too small (need " + std::to_string(L.total) + " bytes)");
            return PO2Q_ERR_WORKSPACE;
        }
        if (!plan_packs_weight(p, h->mode)) continue;  // the conv stages its own weight / reads it as given
        if (!pack_batchable(p, h->mode) || L.nparts > 0) {  // its own pack launch(es), as po2q_qconv2d_pack_f32
            const int st = run_plan(p, nullptr, w[i], nullptr, nullptr, h->bits, h->fsr, h->mode, workspace[i],
                                    workspace_bytes[i], s, ConvEpi{nullptr, nullptr, nullptr, 0}, RUN_PACK);
            if (st) return st;
            continue;
        }
        char* ws = reinterpret_cast<char*>(workspace[i]);
        reqs.push_back(PackReq{&p, w[i], ws + L.packed_off, reinterpret_cast<float*>(ws + L.scale_off), h->bits, h->fsr,
                               h->mode});
        reqs.back().partial = reinterpret_cast<unsigned*>(ws);  // the layout's absmax partials (part_bytes)
    }
    if (reqs.empty()) return PO2Q_OK;
    return hip_status(launch_pack_batch((int)reqs.size(), reqs.data(), s), "batched weight pack launch");
}

int po2q_qconv2d_plan_packs_weight(const po2q_conv_plan* plan) {
    if (!plan) {
        po2q::set_error("po2q: null plan");
        return -PO2Q_ERR_INVALID;
    }
    return plan_packs_weight(plan->p, plan->mode) ? 1 : 0;
}

int po2q_qconv2d_plan_run_packed(const po2q_conv_plan* plan, const float* x, const float* w, const float* bias,
                                 float* y, const float* post_scale, const float* post_shift, const float* residual,
                                 int act, const void* workspace, size_t workspace_bytes, void* stream) {
    using namespace po2q;
    if (!plan || !x || !w || !y || !workspace) {
        set_error("po2q: null plan or pointer");
        return PO2Q_ERR_INVALID;
    }
    if (act < PO2Q_ACT_NONE || act > PO2Q_ACT_SILU) {
        set_error("po2q: unknown activation " + std::to_string(act));
        return PO2Q_ERR_INVALID;
    }
    const ConvEpi e{post_scale, post_shift, residual, act};
    return run_plan(plan->p, x, w, bias, y, plan->bits, plan->fsr, plan->mode, const_cast<void*>(workspace),
                    workspace_bytes, reinterpret_cast<hipStream_t>(stream), e, RUN_CONV);
}

// ------------------------------------------------------------------ inverted-residual block --
// The three plans of one block: expand (optional) 1x1 pointwise, depthwise 3x3 pad 1, project
// 1x1 pointwise, chained shapes, each plan's weight staged in its workspace (the pointwise
// packs and the depthwise plain copy).  Fills the block geometry; 0 or an error with the reason.
static int ir_check(const po2q_conv_plan* e, const po2q_conv_plan* d, const po2q_conv_plan* p, po2q::IrPlan* ip,
                    int64_t* shape) {
    using namespace po2q;
    if (!d || !p) {
        set_error("po2q: inverted residual: null depthwise or project plan");
        return PO2Q_ERR_INVALID;
    }
    auto pointwise = [](const ConvPlan& q) {
        return q.kind == KIND_BF16X3_PW && !q.fp && q.R == 1 && q.S == 1 && q.sh == 1 && q.sw == 1 && q.ph == 0 &&
               q.pw == 0 && q.groups == 1;
    };
    const ConvPlan& D = d->p;
    const ConvPlan& Pj = p->p;
    const int64_t N = D.N, Ch = D.C, H = D.H, W = D.W, S = D.sh;
    std::string why;
    if (D.kind != KIND_DEPTHWISE || D.groups != D.C || D.K != D.C || D.R != 3 || D.S != 3 || D.sh != D.sw ||
        D.ph != 1 || D.pw != 1 || D.dh != 1 || D.dw != 1)
        why = "the depthwise plan is not a 3x3 pad-1 depthwise conv";
    else if (!pointwise(Pj) || Pj.N != N || Pj.C != Ch || Pj.H != D.P || Pj.W != D.Q)
        why = "the project plan is not a pointwise bf16x3 conv of the depthwise output";
    else if (e && (!pointwise(e->p) || e->p.N != N || e->p.K != Ch || e->p.H != H || e->p.W != W))
        why = "the expand plan is not a pointwise bf16x3 conv producing the depthwise input";
    else if ((e && e->mode == PO2Q_MODE_NONE) || d->mode == PO2Q_MODE_NONE || p->mode == PO2Q_MODE_NONE)
        why = "mode none has no staged weights";
    const int64_t Cin = e ? e->p.C : Ch;
    if (why.empty() && !ir_plan(*ip, N, Cin, H, W, Ch, Pj.K, S, e != nullptr))
        why = "no block geometry fits (channels not a multiple of 16, or too large)";
    if (!why.empty()) {
        set_error("po2q: inverted residual: " + why);
        return PO2Q_ERR_UNSUPPORTED;
    }
    if (shape) {
        shape[0] = N; shape[1] = Cin; shape[2] = H; shape[3] = W; shape[4] = Ch; shape[5] = Pj.K; shape[6] = S;
    }
    return PO2Q_OK;
}

int po2q_qconv2d_ir_shape_supported(int64_t N, int64_t Cin, int64_t H, int64_t W, int64_t Ch, int64_t Cout,
                                    int64_t stride, int expand) {
    po2q::IrPlan ip;
    return po2q::ir_plan(ip, N, Cin, H, W, Ch, Cout, stride, expand != 0) ? 1 : 0;
}

int po2q_qconv2d_ir_supported(const po2q_conv_plan* expand, const po2q_conv_plan* depthwise,
                              const po2q_conv_plan* project) {
    po2q::IrPlan ip;
    const int st = ir_check(expand, depthwise, project, &ip, nullptr);
    if (st == PO2Q_OK) return 1;
    return st == PO2Q_ERR_UNSUPPORTED ? 0 : -st;
}

int po2q_qconv2d_ir_f32(const float* x, float* y, const po2q_conv_plan* expand, const void* ws_e, size_t ws_e_bytes,
                        const po2q_conv_plan* depthwise, const void* ws_d, size_t ws_d_bytes,
                        const po2q_conv_plan* project, const void* ws_p, size_t ws_p_bytes, const float* ps1,
                        const float* pb1, int act1, const float* ps2, const float* pb2, int act2, const float* ps3,
                        const float* pb3, const float* residual, int act3, void* stream) {
    using namespace po2q;
    if (!x || !y || !ws_d || !ws_p || (expand && !ws_e)) {
        set_error("po2q: inverted residual: null pointer");
        return PO2Q_ERR_INVALID;
    }
    for (int a : {act1, act2, act3})
        if (a < PO2Q_ACT_NONE || a > PO2Q_ACT_SILU) {
            set_error("po2q: unknown activation " + std::to_string(a));
            return PO2Q_ERR_INVALID;
        }
    IrPlan ip;
    int64_t sh[7];
    int st = ir_check(expand, depthwise, project, &ip, sh);
    if (st) return st;
    const po2q_conv_plan* hs[3] = {expand, depthwise, project};
    const void* wss[3] = {ws_e, ws_d, ws_p};
    const size_t wsb[3] = {ws_e_bytes, ws_d_bytes, ws_p_bytes};
    const char* at[3] = {nullptr, nullptr, nullptr};  // staged weights
    const float* sc[3] = {nullptr, nullptr, nullptr};
    for (int i = 0; i < 3; ++i) {
        if (!hs[i]) continue;
        const WsLayout L = ws_layout(hs[i]->p, hs[i]->mode);
        if (wsb[i] < L.total) {
            set_error("po2q: inverted residual: workspace too small (need " + std::to_string(L.total) + " bytes)");
            return PO2Q_ERR_WORKSPACE;
        }
        at[i] = reinterpret_cast<const char*>(wss[i]) + L.packed_off;
        sc[i] = reinterpret_cast<const float*>(reinterpret_cast<const char*>(wss[i]) + L.scale_off);
    }
    const IrEpi ep{ps1, pb1, ps2, pb2, ps3, pb3, act1, act2, act3, residual};
    return hip_status(launch_conv_ir(ip, x, y, (int)sh[0], (int)sh[1], (int)sh[2], (int)sh[3], (int)sh[4], (int)sh[5],
                                     (int)sh[6], reinterpret_cast<const uint16_t*>(at[0]), sc[0],
                                     reinterpret_cast<const float*>(at[1]), reinterpret_cast<const uint16_t*>(at[2]),
                                     sc[2], ep, reinterpret_cast<hipStream_t>(stream)),
                      "inverted residual launch");
}

int po2q_qconv2d_plan_describe(const po2q_conv_plan* plan, char* buf, size_t len) {
    if (!plan || !buf || len == 0) {
        po2q::set_error("po2q: null plan or buffer");
        return PO2Q_ERR_INVALID;
    }
    describe_plan(plan->p, buf, len);
    return PO2Q_OK;
}

void po2q_qconv2d_plan_destroy(po2q_conv_plan* plan) { delete plan; }
