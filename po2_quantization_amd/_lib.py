"""Python front end of the po2q native library.

The compute path is the PyTorch-ROCm operator library torch.ops.po2q.* (csrc/po2q_torch.cpp,
built into lib/libpo2q_torch.so by build_ext.py on top of the C ABI include/po2q.h): the
quantize / qconv2d / qconv2d_fused / quantize_lin ops validate tensors, keep one resolved
plan handle per conv problem and launch on torch's current HIP stream (they compose with
torch streams and graph capture).  The ctypes binding of the same C ABI below serves the
planning / tuning / diagnostic entry points, the two-enqueue SplitConv, and every call when
PO2Q_LIB points at another build of libpo2q.so (diagnostic builds).

fp32 HIP tensors always run the native kernels: a missing library raises, there is no
torch fallback for them.  The PO2 / PO2+ quantizer also takes fp64 and bf16 HIP tensors natively
(the reference preserves dtype); other inputs (CPU tensors, fp16, ...) take
restated_quantize, the reference formula written as torch ops in the input's dtype and device.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
_DEFAULT_LIB = os.path.join(_HERE, "lib", "libpo2q.so")
LIB_PATH = os.environ.get("PO2Q_LIB", _DEFAULT_LIB)
OPS_PATH = os.path.join(_HERE, "lib", "libpo2q_torch.so")

MODES = {None: 0, "none": 0, "po2": 1, "po2+": 2}
PRECISIONS = {"auto": 0, "fp32": 1, "bf16x3": 2}
# fused epilogue activations (include/po2q.h enum po2q_act)
ACTS = {None: 0, "none": 0, "relu": 1, "relu6": 2, "silu": 3}

# every symbol include/po2q.h declares (checked by tests/test_capi.py)
EXPORTS = (
    "po2q_version",
    "po2q_last_error",
    "po2q_quantize_workspace_bytes",
    "po2q_quantize_f32",
    "po2q_quantize_f64",
    "po2q_quantize_bf16",
    "po2q_quantize_lin_f32",
    "po2q_qconv2d_workspace_bytes",
    "po2q_qconv2d_f32",
    "po2q_qconv2d_fused_f32",
    "po2q_qconv2d_pack_f32",
    "po2q_qconv2d_packed_f32",
    "po2q_qconv2d_autotune",
    "po2q_qconv2d_plans",
    "po2q_qconv2d_f32_plan",
    "po2q_qconv2d_describe",
    "po2q_qconv2d_plan_create",
    "po2q_qconv2d_plan_workspace_bytes",
    "po2q_qconv2d_plan_run",
    "po2q_qconv2d_plan_describe",
    "po2q_qconv2d_plan_destroy",
    "po2q_qconv2d_wgrad_workspace_bytes",
    "po2q_qconv2d_wgrad_f32",
    "po2q_qconv2d_pair_supported",
    "po2q_qconv2d_pair_f32",
    "po2q_qconv2d_s2ds_supported",
    "po2q_qconv2d_s2ds_f32",
    "po2q_qconv2d_plan_pack_batch",
    "po2q_qconv2d_plan_run_packed",
    "po2q_qconv2d_plan_packs_weight",
    "po2q_dilate_f32",
    "po2q_qconv2d_chain_supported",
    "po2q_qconv2d_chain_workspace_bytes",
    "po2q_qconv2d_chain_f32",
    "po2q_qconv2d_ir_supported",
    "po2q_qconv2d_ir_shape_supported",
    "po2q_qconv2d_ir_f32",
)

# Kernel autotuning on the first call per conv problem, the counterpart of
# torch.backends.cudnn.benchmark (reference train.py:33 / test.py:31 set it):
# None follows torch.backends.cudnn.benchmark, True / False force it.
benchmark = None
_tuned = set()
# Optional persistent tuning record (the counterpart of a find-db): with
# PO2Q_TUNE_FILE set, autotuned choices are saved as {problem key: plan index}
# and reused by later processes (same library build, same candidate list).
_tune_file = os.environ.get("PO2Q_TUNE_FILE")
_tune_db = None

_lib = None
_ops = None


class Po2qError(RuntimeError):
    pass


def ops():
    """torch.ops.po2q, loading lib/libpo2q_torch.so once (raises if it has not been built),
    or None when PO2Q_LIB selects another libpo2q build (the ops link the default one)."""
    global _ops
    if _ops is not None:
        return _ops
    if os.path.realpath(LIB_PATH) != os.path.realpath(_DEFAULT_LIB):
        return None
    if not os.path.exists(OPS_PATH):
        raise Po2qError("po2q: operator library %s not found; build it with "
                        "`python -c 'import __graft_entry__ as g; g.build()'`" % OPS_PATH)
    load()  # the same libpo2q.so the ops link (one process-wide plan / tune cache)
    torch.ops.load_library(OPS_PATH)
    _ops = torch.ops.po2q
    return _ops


def _op_call(fn, *args, **kwargs):
    try:
        return fn(*args, **kwargs)
    except RuntimeError as e:  # TORCH_CHECK -> RuntimeError; keep the po2q error type
        raise Po2qError(str(e).split("\nException raised from")[0]) from None


def load():
    """Load libpo2q.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise Po2qError(
            "po2q: native library %s not found; build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` or `make -C po2_quantization_amd/csrc`" % LIB_PATH
        )
    L = ctypes.CDLL(LIB_PATH)
    i64, i32, p, sz = ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t
    L.po2q_version.restype = ctypes.c_char_p
    L.po2q_version.argtypes = []
    L.po2q_last_error.restype = ctypes.c_char_p
    L.po2q_last_error.argtypes = []
    L.po2q_quantize_workspace_bytes.restype = sz
    L.po2q_quantize_workspace_bytes.argtypes = [i64]
    L.po2q_quantize_f32.restype = i32
    L.po2q_quantize_f32.argtypes = [p, p, i64, i32, i32, i32, p, sz, p]
    L.po2q_quantize_lin_f32.restype = i32
    L.po2q_quantize_lin_f32.argtypes = [p, p, i64, i64, i64, i64, i32, i32, i32, p]
    L.po2q_qconv2d_workspace_bytes.restype = sz
    L.po2q_qconv2d_workspace_bytes.argtypes = [i64] * 14 + [i32, i32, i32, i32]
    L.po2q_qconv2d_f32.restype = i32
    L.po2q_qconv2d_f32.argtypes = [p, p, p, p] + [i64] * 14 + [i32, i32, i32, i32, p, sz, p]
    L.po2q_qconv2d_fused_f32.restype = i32
    L.po2q_qconv2d_fused_f32.argtypes = [p, p, p, p] + [i64] * 14 + [i32, i32, i32, i32, p, p, p, i32, p, sz, p]
    L.po2q_qconv2d_pack_f32.restype = i32
    L.po2q_qconv2d_pack_f32.argtypes = [i32, p] + [i64] * 14 + [i32, i32, i32, i32, p, sz, p]
    L.po2q_qconv2d_packed_f32.restype = i32
    L.po2q_qconv2d_packed_f32.argtypes = [i32, p, p, p] + [i64] * 14 + [i32, i32, i32, i32, p, sz, p]
    L.po2q_qconv2d_autotune.restype = i32
    L.po2q_qconv2d_autotune.argtypes = ([p, p, p, p] + [i64] * 14 + [i32, i32, i32, i32, p, sz, p]
                                        + [ctypes.c_char_p, sz])
    L.po2q_qconv2d_plans.restype = i32
    L.po2q_qconv2d_plans.argtypes = [i64] * 14 + [i32] * 5 + [ctypes.c_char_p, sz]
    L.po2q_qconv2d_f32_plan.restype = i32
    L.po2q_qconv2d_f32_plan.argtypes = [i32, p, p, p, p] + [i64] * 14 + [i32, i32, i32, i32, p, sz, p]
    L.po2q_qconv2d_describe.restype = i32
    L.po2q_qconv2d_describe.argtypes = [i64] * 14 + [i32, i32, i32, i32, ctypes.c_char_p, sz]
    L.po2q_qconv2d_pair_supported.restype = i32
    L.po2q_qconv2d_pair_supported.argtypes = [i64] * 4 + [i32] * 3
    L.po2q_qconv2d_s2ds_supported.restype = i32
    L.po2q_qconv2d_s2ds_supported.argtypes = [i64] * 4 + [i32] * 3
    L.po2q_qconv2d_plan_create.restype = i32
    L.po2q_qconv2d_plan_create.argtypes = [ctypes.POINTER(p), i32] + [i64] * 14 + [i32] * 4
    L.po2q_qconv2d_plan_workspace_bytes.restype = sz
    L.po2q_qconv2d_plan_workspace_bytes.argtypes = [p]
    L.po2q_qconv2d_plan_destroy.restype = None
    L.po2q_qconv2d_plan_destroy.argtypes = [p]
    L.po2q_qconv2d_plan_pack_batch.restype = i32
    L.po2q_qconv2d_plan_pack_batch.argtypes = [i32, ctypes.POINTER(p), ctypes.POINTER(p), ctypes.POINTER(p),
                                               ctypes.POINTER(sz), p]
    L.po2q_qconv2d_plan_run_packed.restype = i32
    L.po2q_qconv2d_plan_run_packed.argtypes = [p] * 8 + [i32, p, sz, p]
    L.po2q_qconv2d_plan_packs_weight.restype = i32
    L.po2q_qconv2d_plan_packs_weight.argtypes = [p]
    L.po2q_qconv2d_ir_supported.restype = i32
    L.po2q_qconv2d_ir_supported.argtypes = [p, p, p]
    L.po2q_qconv2d_ir_shape_supported.restype = i32
    L.po2q_qconv2d_ir_shape_supported.argtypes = [i64] * 7 + [i32]
    L.po2q_qconv2d_ir_f32.restype = i32
    L.po2q_qconv2d_ir_f32.argtypes = [p, p, p, p, sz, p, p, sz, p, p, sz, p, p, i32, p, p, i32, p, p, p, i32, p]
    L.po2q_qconv2d_chain_supported.restype = i32
    L.po2q_qconv2d_chain_supported.argtypes = [i64] * 4 + [i32] * 4
    L.po2q_qconv2d_chain_workspace_bytes.restype = sz
    L.po2q_qconv2d_chain_workspace_bytes.argtypes = [i64] * 4 + [i32]
    L.po2q_qconv2d_chain_f32.restype = i32
    L.po2q_qconv2d_chain_f32.argtypes = ([p] * 7 + [i32] + [i64] * 4 + [i32] * 3 + [p, p, sz, p])
    _lib = L
    return L


def _check(status):
    if status != 0:
        raise Po2qError(load().po2q_last_error().decode())


def _require_hip_f32(t, what):
    if not isinstance(t, torch.Tensor):
        raise TypeError("po2q: %s must be a torch.Tensor" % what)
    if t.device.type != "cuda":
        raise Po2qError("po2q: %s must be a HIP device tensor (got %s); the po2q ops have no CPU path"
                        % (what, t.device))
    if t.dtype != torch.float32:
        raise Po2qError("po2q: %s must be float32 (got %s)" % (what, t.dtype))


def _stream(dev):
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def _workspace(nbytes, dev):
    return torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=dev)


def restated_quantize(w, bits, mode, fsr=1):
    """PO2 / PO2+ for inputs the native kernels do not take (CPU tensors; fp16 and other dtypes on
    the GPU): the reference's elementwise formula (utils/quantizers.py:21-32, :41-52) as torch ops in
    w's own dtype and device, so torch's log2 / round of that device decide.  On CPU tensors that is
    the reference's own arithmetic: bit for bit its outputs in every dtype
    (tests/test_restated_quantizer.py).  fp32, fp64 and bf16 HIP tensors take the native kernels,
    bit-exact with the reference's CPU results (tests/test_gpu_quantizer.py)."""
    scale = torch.max(torch.abs(w))  # (raises for an empty tensor, as the reference does)
    a = (w / scale).abs()
    t = torch.log2(a / 1.5) + 0.5 if mode == "po2+" else torch.log2(a)
    lo, hi = fsr - 2 ** (bits - 1), fsr - 1
    e = torch.clamp(torch.round(t), lo, hi)
    # 2**e from a table of exact powers of two (Python floats are exact): a device's
    # pow(2, e) need not be (it is not for fp64 on the GPU), the CPU reference's is
    levels = torch.tensor([2.0 ** k for k in range(lo, hi + 1)], dtype=w.dtype, device=w.device)
    nan = torch.isnan(e)
    # (a bf16 clamp bound below -256 is itself rounded, e.g. -2047 -> -2048: such e are far below
    # bf16's range, 2**e == 0 either way, so the index is clamped into the table)
    p2 = levels[(torch.where(nan, lo, e).long() - lo).clamp(0, hi - lo)]
    p2 = torch.where(nan, e, p2)
    return p2 * torch.sign(w) * scale


def quantize(w, bits, mode, fsr=1):
    """PO2 / PO2+ quantization of a whole tensor (utils/quantizers.py:19-56)."""
    if not isinstance(w, torch.Tensor):
        raise TypeError("po2q: input must be a torch.Tensor")
    mode_id = MODES[mode]
    if mode_id == 0:
        raise Po2qError("po2q: quantize() needs mode 'po2' or 'po2+'")
    native = w.device.type == "cuda" and w.dtype in (torch.float32, torch.float64, torch.bfloat16)
    if not native:
        return restated_quantize(w, int(bits), mode, int(fsr))
    if w.numel() == 0:
        raise Po2qError("po2q: max(): Expected reduction dim to be specified for input.numel() == 0")
    O = ops()
    if O is not None:
        return _op_call(O.quantize, w, int(bits), mode_id, int(fsr))
    if w.dtype != torch.float32:
        raise Po2qError("po2q: fp64 / bf16 quantize needs the operator library (PO2Q_LIB selects another build)")
    L = load()
    wc = w.contiguous()
    out = torch.empty_like(wc)
    n = wc.numel()
    with torch.cuda.device(wc.device):
        ws = _workspace(L.po2q_quantize_workspace_bytes(n), wc.device)
        _check(L.po2q_quantize_f32(wc.data_ptr(), out.data_ptr(), n, int(bits), int(fsr), mode_id,
                                   ws.data_ptr(), ws.numel(), _stream(wc.device)))
    return out


def restated_quantize_lin(w, bits, plus, num_iters=10):
    """lin / lin+ for CPU tensors: the reference's per-input-channel refit (utils/quantizers.py:8-16,
    59-136) as the same torch ops in the same order, so on CPU it is the reference's own arithmetic.
    The channel axis is dim 1; its step broadcasts over (C, R, S) as the reference's view(-1, 1, 1)."""
    if w.dim() != 4:
        raise Po2qError("po2q: the lin quantizers need a 4-D weight (got %d dims)" % w.dim())
    top = 2 ** (bits - 1) - 1

    def snap(step):  # quantize_per_filter(w, step, bits) / step
        s = step.view(-1, 1, 1)
        return (s * torch.clamp(torch.round(w / s), min=-top, max=top)) / s

    hi = w.max(dim=3).values.max(dim=2).values.max(dim=0).values
    lo = w.min(dim=3).values.min(dim=2).values.min(dim=0).values
    step = (hi - lo) / (2 ** bits - 1)
    q = snap(step)
    shrink = torch.sqrt(torch.tensor(8.0 / 9.0)) if plus else None
    for _ in range(num_iters):
        step = torch.sum(q * w, dim=[0, 2, 3]) / torch.sum(q * q, dim=[0, 2, 3])
        step = 2 ** torch.round(torch.log2(shrink * step if plus else step))
        q = snap(step)
    return q * step.view(-1, 1, 1)


def quantize_lin(w, bits, plus, num_iters=10):
    """lin / lin+ quantization of a 4-D weight, per input channel (dim 1)
    (utils/quantizers.py:59-136).  CPU tensors take restated_quantize_lin."""
    if isinstance(w, torch.Tensor) and not w.is_cuda:
        return restated_quantize_lin(w, int(bits), plus, int(num_iters))
    _require_hip_f32(w, "input")
    if w.dim() != 4:
        # the reference reduces dims 3, 2, 0 explicitly (torch.max(..., dim=3) ...)
        raise Po2qError("po2q: the lin quantizers need a 4-D weight (got %d dims)" % w.dim())
    O = ops()
    if O is not None:
        return _op_call(O.quantize_lin, w, int(bits), int(num_iters), 1 if plus else 0)
    L = load()
    wc = w.contiguous()
    out = torch.empty_like(wc)
    with torch.cuda.device(wc.device):
        _check(L.po2q_quantize_lin_f32(wc.data_ptr(), out.data_ptr(), *wc.shape, int(bits), int(num_iters),
                                       1 if plus else 0, _stream(wc.device)))
    return out


def _pair(v):
    return (int(v), int(v)) if isinstance(v, int) else (int(v[0]), int(v[1]))


def _conv_geometry(x, w, bias, stride, padding, dilation, groups):
    """Validate a conv call like torch's F.conv2d; returns (x, w, bias) contiguous,
    the 14 geometry arguments of the C ABI and the output size."""
    _require_hip_f32(x, "input")
    _require_hip_f32(w, "weight")
    if bias is not None:
        _require_hip_f32(bias, "bias")
    if x.dim() != 4 or w.dim() != 4:
        raise Po2qError("po2q: expected 4-D input and weight, got %d-D and %d-D" % (x.dim(), w.dim()))
    if x.device != w.device or (bias is not None and bias.device != x.device):
        raise Po2qError("po2q: input, weight and bias must be on the same device")
    N, C, H, W = x.shape
    K, Cg, R, S = w.shape
    if Cg * groups != C:
        raise Po2qError("po2q: Given groups=%d, weight of size %s, expected input%s to have %d channels, but got "
                        "%d channels instead" % (groups, list(w.shape), list(x.shape), Cg * groups, C))
    sh, sw = _pair(stride)
    ph, pw = _pair(padding)
    dh, dw = _pair(dilation)
    P = (H + 2 * ph - dh * (R - 1) - 1) // sh + 1
    Q = (W + 2 * pw - dw * (S - 1) - 1) // sw + 1
    args = (N, C, H, W, K, R, S, sh, sw, ph, pw, dh, dw, int(groups))
    bc = bias.contiguous() if bias is not None else None
    return x.contiguous(), w.contiguous(), bc, args, (N, K, max(P, 0), max(Q, 0))


def qconv2d(x, w, bias=None, stride=1, padding=0, dilation=1, groups=1, bits=4, mode="po2", fsr=1,
            precision="auto", plan=None):
    """Fused quantize + conv forward (models/quantized_conv.py:32-38); NCHW fp32 in/out.

    plan=None runs the tuned (or heuristic) plan, autotuning first when benchmark
    mode is on; plan=i runs candidate i of plans() (tests / tuning tools)."""
    xc, wc, bc, args, yshape = _conv_geometry(x, w, bias, stride, padding, dilation, groups)
    mode_id = MODES[mode]
    prec = PRECISIONS[precision]
    if yshape[0] == 0:  # an empty batch: torch's F.conv2d returns an empty output
        return torch.empty(yshape, dtype=torch.float32, device=xc.device)
    O = ops()
    if O is not None:
        key = args + (int(bits), int(fsr), mode_id, prec)
        idx, tune = _plan_choice(key, plan)
        y = _op_call(O.qconv2d, xc, wc, bc, list(args[7:9]), list(args[9:11]), list(args[11:13]), args[13],
                     int(bits), mode_id, int(fsr), prec, idx, tune)
        if tune:
            _after_tune(key)
        return y
    L = load()
    with torch.cuda.device(xc.device):
        nbytes = L.po2q_qconv2d_workspace_bytes(*args, int(bits), int(fsr), mode_id, prec)
        if nbytes == 0:
            _check(1)
        y = torch.empty(yshape, dtype=torch.float32, device=xc.device)
        ws = _workspace(nbytes, xc.device)
        bp = bc.data_ptr() if bc is not None else None
        key = args + (int(bits), int(fsr), mode_id, prec)
        if plan is not None:
            _check(L.po2q_qconv2d_f32_plan(int(plan), xc.data_ptr(), wc.data_ptr(), bp, y.data_ptr(), *key,
                                           ws.data_ptr(), ws.numel(), _stream(xc.device)))
        elif _saved_plan(key) is not None:
            _check(L.po2q_qconv2d_f32_plan(_saved_plan(key), xc.data_ptr(), wc.data_ptr(), bp, y.data_ptr(), *key,
                                           ws.data_ptr(), ws.numel(), _stream(xc.device)))
        elif key not in _tuned and _benchmark_enabled():
            buf = ctypes.create_string_buffer(512)
            _check(L.po2q_qconv2d_autotune(xc.data_ptr(), wc.data_ptr(), bp, y.data_ptr(), *key,
                                           ws.data_ptr(), ws.numel(), _stream(xc.device), buf, 512))
            _tuned.add(key)
            _save_plan(key, buf.value.decode())
        else:
            _check(L.po2q_qconv2d_f32(xc.data_ptr(), wc.data_ptr(), bp, y.data_ptr(), *key,
                                      ws.data_ptr(), ws.numel(), _stream(xc.device)))
    return y


def qconv2d_fused(x, w, bias=None, stride=1, padding=0, dilation=1, groups=1, bits=4, mode="po2", fsr=1,
                  precision="auto", post_scale=None, post_shift=None, residual=None, act="none"):
    """Quantize + conv + eval epilogue in one native call (po2q_qconv2d_fused_f32):
        y = act((conv(x, Q(w)) + bias) * post_scale[k] + post_shift[k] + residual)
    post_scale / post_shift: [K] (an eval BatchNorm folded by the caller) or None;
    residual: a tensor of y's shape or None; act: "none" | "relu" | "relu6" | "silu"."""
    xc, wc, bc, args, yshape = _conv_geometry(x, w, bias, stride, padding, dilation, groups)
    L = load()
    mode_id = MODES[mode]
    prec = PRECISIONS[precision]
    ext = []
    for t, what in ((post_scale, "post_scale"), (post_shift, "post_shift")):
        if t is not None:
            _require_hip_f32(t, what)
            if t.device != xc.device:
                raise Po2qError("po2q: %s must be on the input's device" % what)
            if t.numel() != yshape[1]:
                raise Po2qError("po2q: %s must have %d elements, got %d" % (what, yshape[1], t.numel()))
            t = t.contiguous()
        ext.append(t)
    rc = None
    if residual is not None:
        _require_hip_f32(residual, "residual")
        if residual.device != xc.device:
            raise Po2qError("po2q: residual must be on the input's device")
        if tuple(residual.shape) != tuple(yshape):
            raise Po2qError("po2q: residual shape %s does not match the output %s"
                            % (list(residual.shape), list(yshape)))
        rc = residual.contiguous()
    if yshape[0] == 0:
        return torch.empty(yshape, dtype=torch.float32, device=xc.device)
    O = ops()
    if O is not None:
        # the saved / tuned plan, exactly as qconv2d runs it (autotuning first if due)
        key = args + (int(bits), int(fsr), mode_id, prec)
        idx, tune = _plan_choice(key, None)
        y = _op_call(O.qconv2d_fused, xc, wc, bc, list(args[7:9]), list(args[9:11]), list(args[11:13]), args[13],
                     int(bits), mode_id, int(fsr), prec, idx, tune, ext[0], ext[1], rc, ACTS[act])
        if tune:
            _after_tune(key)
        return y
    with torch.cuda.device(xc.device):
        key = args + (int(bits), int(fsr), mode_id, prec)
        nbytes = L.po2q_qconv2d_workspace_bytes(*key)
        if nbytes == 0:
            _check(1)
        if key not in _tuned and _saved_plan(key) is None and _benchmark_enabled():
            qconv2d(xc, wc, bc, stride, padding, dilation, groups, bits, mode, fsr, precision)  # autotune once
        y = torch.empty(yshape, dtype=torch.float32, device=xc.device)
        ws = _workspace(nbytes, xc.device)
        ptr = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
        _check(L.po2q_qconv2d_fused_f32(xc.data_ptr(), wc.data_ptr(), ptr(bc), y.data_ptr(), *key,
                                        ptr(ext[0]), ptr(ext[1]), ptr(rc), ACTS[act],
                                        ws.data_ptr(), ws.numel(), _stream(xc.device)))
    return y


class SplitConv:
    """One quantized conv layer as two enqueues (po2q_qconv2d_pack_f32 /
    po2q_qconv2d_packed_f32): the weight quantize + pack into a workspace this object
    owns, then the conv from it.  pack() may run on another stream than conv(); the
    caller orders them (events) and must not re-pack while a conv still reads the
    workspace.  The plan is the one qconv2d() runs for these arguments (call qconv2d
    once first when autotuning)."""

    def __init__(self, x_shape, w, stride=1, padding=0, dilation=1, groups=1, bits=4, mode="po2", fsr=1,
                 precision="auto"):
        _require_hip_f32(w, "weight")
        N, C, H, W = (int(v) for v in x_shape)
        K, Cg, R, S = w.shape
        sh, sw = _pair(stride)
        ph, pw = _pair(padding)
        dh, dw = _pair(dilation)
        self.w = w.contiguous()
        self.key = (N, C, H, W, K, R, S, sh, sw, ph, pw, dh, dw, int(groups), int(bits), int(fsr), MODES[mode],
                    PRECISIONS[precision])
        P = (H + 2 * ph - dh * (R - 1) - 1) // sh + 1
        Q = (W + 2 * pw - dw * (S - 1) - 1) // sw + 1
        self.yshape = (N, K, P, Q)
        L = load()
        nbytes = L.po2q_qconv2d_workspace_bytes(*self.key)
        if nbytes == 0:
            _check(1)
        self.ws = _workspace(nbytes, w.device)

    def _plan(self):
        idx = _saved_plan(self.key)
        return -1 if idx is None else int(idx)

    def pack(self, stream=None):
        s = stream if stream is not None else torch.cuda.current_stream(self.w.device)
        _check(load().po2q_qconv2d_pack_f32(self._plan(), self.w.data_ptr(), *self.key, self.ws.data_ptr(),
                                            self.ws.numel(), ctypes.c_void_p(s.cuda_stream)))

    def conv(self, x, bias=None):
        _require_hip_f32(x, "input")
        if tuple(x.shape) != tuple(self.key[:4]):
            raise Po2qError("po2q: input shape %s does not match the packed layer's %s"
                            % (list(x.shape), list(self.key[:4])))
        xc = x.contiguous()
        y = torch.empty(self.yshape, dtype=torch.float32, device=xc.device)
        bp = bias.contiguous().data_ptr() if bias is not None else None
        _check(load().po2q_qconv2d_packed_f32(self._plan(), xc.data_ptr(), bp, y.data_ptr(), *self.key,
                                              self.ws.data_ptr(), self.ws.numel(), _stream(xc.device)))
        return y


def pair_supported(x_shape, bits=4, mode="po2", fsr=1):
    """True when qconv2d_pair takes this input shape (16 or 32 channels, W % 4 == 0, W <= 224
    / 112, po2 / po2+ with the exponent window inside bf16's range) and is the faster path
    (C = 16 with W >= 128; elsewhere two single-conv calls measured faster)."""
    if mode not in ("po2", "po2+"):
        return False
    N, C, H, W = (int(v) for v in x_shape)
    return bool(load().po2q_qconv2d_pair_supported(N, C, H, W, int(bits), int(fsr), MODES[mode]))


def qconv2d_pair(x, w1, w2, bits=4, mode="po2", fsr=1, bias1=None, bias2=None, post_scale1=None, post_shift1=None,
                 act1="none", post_scale2=None, post_shift2=None, residual=None, act2="none"):
    """Two chained quantized 3x3 / stride-1 / pad-1 convs (C -> C -> C channels, C = 16 or 32)
    in one launch (po2q_qconv2d_pair_f32), the intermediate kept on chip:
        h = act1((conv(x, Q(w1)) + bias1) * post_scale1 + post_shift1)
        y = act2((conv(h, Q(w2)) + bias2) * post_scale2 + post_shift2 + residual)
    -- qconv2d_fused twice, as a ResNet56 stage-1 / stage-2 BasicBlock chains them (resnet.py:55-71)."""
    for t, what in ((x, "input"), (w1, "weight1"), (w2, "weight2")):
        _require_hip_f32(t, what)
    O = ops()
    if O is None:
        raise Po2qError("po2q: qconv2d_pair needs the operator library (PO2Q_LIB selects another build)")
    return _op_call(O.qconv2d_pair, x, w1, w2, int(bits), MODES[mode], int(fsr), bias1, bias2, post_scale1,
                    post_shift1, ACTS[act1], post_scale2, post_shift2, residual, ACTS[act2])


CHAIN_MAX_LAYERS = 24  # include/po2q.h PO2Q_CHAIN_MAX_LAYERS


def chain_supported(x_shape, n_layers, bits=4, mode="po2", fsr=1):
    """Whether qconv2d_chain takes n_layers C -> C 3x3 / stride-1 convs on x of this shape
    (po2q_qconv2d_chain_supported: C in {16, 32, 64}, W % 4 == 0, the padded image's split planes
    in LDS -- CIFAR sizes)."""
    N, C, H, W = (int(v) for v in x_shape)
    return bool(load().po2q_qconv2d_chain_supported(N, C, H, W, int(n_layers), int(bits), int(fsr),
                                                     MODES[mode]))


def qconv2d_chain(x, weights, bits=4, mode="po2", fsr=1, biases=None, post_scales=None, post_shifts=None,
                  acts=None, res_from=None):
    """len(weights) quantized 3x3 / stride-1 / pad-1 C -> C convs in ONE launch (po2q_qconv2d_chain_f32,
    torch.ops.po2q.qconv2d_chain):
        a_0 = x;  a_{l+1} = act_l((conv(a_l, Q(w_l)) + bias_l) * post_scale_l + post_shift_l
                                  (+ a_{res_from[l]}));   returns a_L
    -- the stride-1 run of a ResNet stage at CIFAR size, QuantizedConv2d.forward after
    QuantizedConv2d.forward as models/resnet.py:55-71 chains them (BN folded into the affine, the
    identity shortcut as res_from = the block's first layer).  A None list: none for every layer;
    a None entry: none for that layer; a list must have one entry per weight."""
    n = len(weights)
    for what, lst in (("biases", biases), ("post_scales", post_scales), ("post_shifts", post_shifts),
                      ("acts", acts), ("res_from", res_from)):
        if lst is not None and len(lst) != n:
            raise Po2qError("po2q: chain: %s must have one entry per weight (%d), got %d" % (what, n, len(lst)))
    _require_hip_f32(x, "input")
    for i, w in enumerate(weights):
        _require_hip_f32(w, "weight %d" % i)
    O = ops()
    if O is not None:
        return _op_call(O.qconv2d_chain, x, list(weights), int(bits), MODES[mode], int(fsr),
                        list(biases) if biases is not None else [], list(post_scales) if post_scales is not None else [],
                        list(post_shifts) if post_shifts is not None else [],
                        [ACTS[a] for a in acts] if acts is not None else [],
                        [-1 if r is None else int(r) for r in res_from] if res_from is not None else [])
    L = load()
    xc = x.contiguous()
    N, C, H, W = (int(v) for v in xc.shape)
    ws_ = [w.contiguous() for w in weights]
    for i, w in enumerate(ws_):
        if tuple(w.shape) != (C, C, 3, 3):
            raise Po2qError("po2q: chain weight %d must be [%d, %d, 3, 3], got %s" % (i, C, C, tuple(w.shape)))

    def ptrs(ts, what):
        if ts is None:
            return None, []
        keep = []
        arr = (ctypes.c_void_p * n)()
        for i, t in enumerate(ts):
            if t is None:
                arr[i] = None
                continue
            _require_hip_f32(t, "%s %d" % (what, i))
            tc = t.contiguous()
            if tc.numel() != C:
                raise Po2qError("po2q: chain %s %d must have %d elements" % (what, i, C))
            keep.append(tc)
            arr[i] = tc.data_ptr()
        return arr, keep

    wa = (ctypes.c_void_p * n)(*[w.data_ptr() for w in ws_])
    ba, kb = ptrs(biases, "bias")
    sa, ks = ptrs(post_scales, "post_scale")
    ha, kh = ptrs(post_shifts, "post_shift")
    aa = (ctypes.c_int * n)(*[ACTS[a] for a in acts]) if acts is not None else None
    ra = (ctypes.c_int * n)(*[-1 if r is None else int(r) for r in res_from]) if res_from is not None else None
    y = torch.empty_like(xc)
    nbytes = L.po2q_qconv2d_chain_workspace_bytes(N, C, H, W, n)
    ws = _workspace(nbytes, xc.device)
    _check(L.po2q_qconv2d_chain_f32(xc.data_ptr(), wa, ba, sa, ha, aa, ra, n, N, C, H, W, int(bits), int(fsr),
                                    MODES[mode], y.data_ptr(), ws.data_ptr(), max(int(nbytes), 256),
                                    _stream(xc.device)))
    return y


def _layer_geometry(x_shape, stride, padding, dilation, groups):
    """The 11 geometry ints of qconv2d_pack_batch for one layer: N C H W, stride, padding, dilation, groups."""
    N, C, H, W = (int(v) for v in x_shape)
    return [N, C, H, W, *_pair(stride), *_pair(padding), *_pair(dilation), int(groups)]


def pack_batch(layers, bits=4, mode="po2", fsr=1, precision="auto", plans=None):
    """The weight quantize + pack of several QuantizedConv2d.forward calls (models/quantized_conv.py:35)
    as batched launches (torch.ops.po2q.qconv2d_pack_batch -> po2q_qconv2d_plan_pack_batch): layers =
    [(w, x_shape, stride, padding, dilation, groups)], all with this (bits, mode, fsr, precision).
    Returns one workspace per layer for qconv2d_packed (an empty one where the layer's kernel stages
    its own weight).  Every layer runs the plan qconv2d() would run for it (the tuned / saved one), or
    plans[i] when given and not None (a candidate index, as qconv2d_packed(plan=) / qconv2d_ir take)."""
    O = ops()
    if O is None:
        raise Po2qError("po2q: pack_batch needs the operator library (PO2Q_LIB selects another build)")
    mode_id, prec = MODES[mode], PRECISIONS[precision]
    geom, plans_, ws = [], [], []
    if plans is not None and len(plans) != len(layers):
        raise Po2qError("po2q: pack_batch: one plan per layer (or none)")
    for i, (w, x_shape, stride, padding, dilation, groups) in enumerate(layers):
        _require_hip_f32(w, "weight")
        g = _layer_geometry(x_shape, stride, padding, dilation, groups)
        geom += g
        if plans is not None and plans[i] is not None:
            plans_.append(int(plans[i]))
        else:
            K, _, R, S = w.shape
            key = tuple(g[:4]) + (int(K), int(R), int(S)) + tuple(g[4:]) + (int(bits), int(fsr), mode_id, prec)
            saved = _saved_plan(key)
            plans_.append(-1 if saved is None else int(saved))
        ws.append(w)
    return _op_call(O.qconv2d_pack_batch, ws, geom, int(bits), mode_id, int(fsr), prec, plans_)


def qconv2d_packed(x, w, workspace, bias=None, stride=1, padding=0, dilation=1, groups=1, bits=4, mode="po2", fsr=1,
                   precision="auto", post_scale=None, post_shift=None, residual=None, act="none", plan=None):
    """qconv2d_fused from a workspace pack_batch filled (the conv and its epilogue only; the weight
    was quantized + packed by the batched launch).  Bit for bit qconv2d_fused's result.  plan: the
    candidate index the workspace was packed for (None: the tuned / saved plan, as pack_batch)."""
    O = ops()
    if O is None:
        raise Po2qError("po2q: qconv2d_packed needs the operator library (PO2Q_LIB selects another build)")
    xc, wc, bc, args, yshape = _conv_geometry(x, w, bias, stride, padding, dilation, groups)
    key = args + (int(bits), int(fsr), MODES[mode], PRECISIONS[precision])
    saved = _saved_plan(key) if plan is None else int(plan)
    return _op_call(O.qconv2d_packed, xc, wc, workspace, bc, list(args[7:9]), list(args[9:11]), list(args[11:13]),
                    args[13], int(bits), MODES[mode], int(fsr), PRECISIONS[precision], -1 if saved is None else int(saved),
                    post_scale, post_shift, residual, ACTS[act])


def ir_shape_supported(x_shape, Ch, Cout, stride, expand):
    """Whether the fused inverted-residual kernel takes this block by default (po2q_qconv2d_ir_shape_supported:
    where it measured faster than the three layer launches).  Host-only."""
    N, Cin, H, W = (int(v) for v in x_shape)
    return load().po2q_qconv2d_ir_shape_supported(N, Cin, H, W, int(Ch), int(Cout), int(stride), int(bool(expand))) == 1


def qconv2d_ir(x, we, wd, wp, ws_e, ws_d, ws_p, stride=1, bits=4, mode="po2", fsr=1, precision="auto",
               ps1=None, pb1=None, act1="relu6", ps2=None, pb2=None, act2="relu6", ps3=None, pb3=None,
               residual=None, act3="none", plans=(0, 0, 0)):
    """One inverted-residual block (reference mobilenet.py:53-134: expand 1x1 -> BN -> act ->
    depthwise 3x3 -> BN -> act -> project 1x1 -> BN (+ x); we = None: no expand) in ONE launch
    (torch.ops.po2q.qconv2d_ir -> po2q_qconv2d_ir_f32) from the three layers' workspaces filled by
    pack_batch (ws_e None without expand).  The hidden activations stay on chip; the result is the
    three qconv2d_packed calls' up to the pointwise kernels' k-split summation order.  Shapes the
    fused kernel does not take run as those three calls.  plans: the candidate index each workspace was
    packed for (pack_batch(plans=)); the default 0 is each layer's heuristic plan (the pointwise and
    depthwise kernels whose packs the block kernel reads), None entries the tuned / saved plan."""
    O = ops()
    if O is None:
        raise Po2qError("po2q: qconv2d_ir needs the operator library (PO2Q_LIB selects another build)")
    _require_hip_f32(x, "input")
    N, Cin, H, W = (int(v) for v in x.shape)
    Ch, Cout, s = int(wd.shape[0]), int(wp.shape[0]), int(stride)
    Ho, Wo = (H - 1) // s + 1, (W - 1) // s + 1
    mode_id, prec = MODES[mode], PRECISIONS[precision]
    tail = (int(bits), int(fsr), mode_id, prec)
    keys = [(N, Cin, H, W, Ch, 1, 1, 1, 1, 0, 0, 1, 1, 1) + tail if we is not None else None,
            (N, Ch, H, W, Ch, 3, 3, s, s, 1, 1, 1, 1, Ch) + tail,
            (N, Ch, Ho, Wo, Cout, 1, 1, 1, 1, 0, 0, 1, 1, 1) + tail]
    plans_ = []
    for k, pl in zip(keys, plans):
        saved = (_saved_plan(k) if k is not None else None) if pl is None else pl
        plans_.append(-1 if saved is None else int(saved))
    return _op_call(O.qconv2d_ir, x, we, wd, wp, ws_e, ws_d, ws_p, s, int(bits), mode_id, int(fsr), prec, ps1, pb1,
                    ACTS[act1], ps2, pb2, ACTS[act2], ps3, pb3, residual, ACTS[act3], plans_)


class PackedConvs:
    """Several QuantizedConv2d forwards (models/quantized_conv.py:32-38) with their weight
    quantize + pack as ONE batched launch (po2q_qconv2d_plan_pack_batch) and each conv from its
    packed workspace (po2q_qconv2d_plan_run_packed) -- the same kernels and results as
    qconv2d() layer by layer, with ceil(n / 36) pack launches instead of one per layer.

    specs: [(x_shape, w, stride, padding)] in call order (groups 1, dilation 1, no bias); the
    plans are resolved once here, so create it after the shapes were autotuned.  Call pack()
    once per forward (after any weight update), then conv(i, x) for each layer.

    w is a weight tensor or a module with a .weight (a QuantizedConv2d).  A module's .weight is
    re-read at every pack() and conv(), so a replaced parameter (load_state_dict(assign=True),
    module.weight = ..., .to()) is picked up; a tensor is held by reference and must be updated in
    place (pack() raises if its storage changed)."""

    def __init__(self, specs, bits=4, mode="po2", fsr=1):
        L = load()
        self._L = L
        self.bits, self.mode, self.fsr = int(bits), MODES[mode], int(fsr)
        self.plans, self.ws, self.w, self.xshape, self.yshape = [], [], [], [], []
        self.src = []
        for x_shape, w, stride, padding in specs:
            self.src.append(w)
            w = w.weight if hasattr(w, "weight") and not isinstance(w, torch.Tensor) else w
            _require_hip_f32(w, "weight")
            if not w.is_contiguous():
                raise Po2qError("po2q: PackedConvs needs contiguous weights (it reads them in place at every pack)")
            N, C, H, W = (int(v) for v in x_shape)
            K, _, R, S = w.shape
            sh, sw = _pair(stride)
            ph, pw = _pair(padding)
            args = (N, C, H, W, K, R, S, sh, sw, ph, pw, 1, 1, 1)
            key = args + (self.bits, self.fsr, self.mode, 0)
            saved = _saved_plan(key)
            h = ctypes.c_void_p()
            _check(L.po2q_qconv2d_plan_create(ctypes.byref(h), -1 if saved is None else int(saved), *args,
                                              self.bits, self.fsr, self.mode, 0))
            self.plans.append(h)
            self.ws.append(_workspace(L.po2q_qconv2d_plan_workspace_bytes(h), w.device))
            self.w.append(w)
            self.xshape.append((N, C, H, W))
            self.yshape.append((N, K, (H + 2 * ph - R) // sh + 1, (W + 2 * pw - S) // sw + 1))
        n = len(self.plans)
        self._n = n
        self._pa = (ctypes.c_void_p * n)(*[h.value for h in self.plans])
        self._wptr = [w.data_ptr() for w in self.w]
        self._wa = (ctypes.c_void_p * n)(*self._wptr)
        self._sa = (ctypes.c_void_p * n)(*[t.data_ptr() for t in self.ws])
        self._ba = (ctypes.c_size_t * n)(*[t.numel() for t in self.ws])

    def _refresh(self):
        """Re-read the modules' weights; returns False if nothing changed."""
        changed = False
        for i, src in enumerate(self.src):
            if isinstance(src, torch.Tensor):
                if src.data_ptr() != self._wptr[i]:
                    raise Po2qError("po2q: PackedConvs weight %d changed storage since construction "
                                    "(set_() / resize); pass the module instead, or build a new PackedConvs" % i)
                continue
            w = src.weight
            if w is self.w[i] and w.data_ptr() == self._wptr[i]:
                continue
            _require_hip_f32(w, "weight")
            if tuple(w.shape) != tuple(self.w[i].shape) or w.device != self.w[i].device or not w.is_contiguous():
                raise Po2qError("po2q: PackedConvs module %d's weight changed shape / device / layout; build a new "
                                "PackedConvs" % i)
            self.w[i] = w
            self._wptr[i] = w.data_ptr()
            self._wa[i] = w.data_ptr()
            changed = True
        return changed

    def pack(self):
        self._refresh()
        if self._n:
            _check(self._L.po2q_qconv2d_plan_pack_batch(self._n, self._pa, self._wa, self._sa, self._ba,
                                                        _stream(self.w[0].device)))

    def conv(self, i, x):
        _require_hip_f32(x, "input")
        if tuple(x.shape) != self.xshape[i]:
            raise Po2qError("po2q: PackedConvs layer %d was planned for input %s, got %s"
                            % (i, self.xshape[i], tuple(x.shape)))
        x = x.contiguous()
        y = torch.empty(self.yshape[i], dtype=torch.float32, device=x.device)
        ws = self.ws[i]
        _check(self._L.po2q_qconv2d_plan_run_packed(self.plans[i], x.data_ptr(), self.w[i].data_ptr(), None,
                                                    y.data_ptr(), None, None, None, 0, ws.data_ptr(), ws.numel(),
                                                    _stream(x.device)))
        return y

    def __del__(self):
        L = getattr(self, "_L", None)
        for h in getattr(self, "plans", []):
            if L is not None and h:
                L.po2q_qconv2d_plan_destroy(h)


def s2ds_supported(x_shape, bits=4, mode="po2", fsr=1):
    """True when qconv2d_s2ds takes this input shape (C = 16 or 32 -> 2C, W % 4 == 0, po2 / po2+).
    PO2Q_S2DS=0 turns the fused transition off (A/B runs)."""
    if mode not in ("po2", "po2+") or os.environ.get("PO2Q_S2DS") == "0":
        return False
    N, C, H, W = (int(v) for v in x_shape)
    return bool(load().po2q_qconv2d_s2ds_supported(N, C, H, W, int(bits), int(fsr), MODES[mode]))


def qconv2d_s2ds(x, w, wds, bits=4, mode="po2", fsr=1, post_scale=None, post_shift=None, act="none",
                 post_scale_ds=None, post_shift_ds=None):
    """A stage's stride-2 transition in one launch (po2q_qconv2d_s2ds_f32): the 3x3 stride-2 conv1 and
    the 1x1 stride-2 projection shortcut of the first BasicBlock (reference resnet.py:55-71, each a
    QuantizedConv2d.forward, quantized_conv.py:32-38) on the same x, which is read once:
        y   = act(conv(x, Q(w), stride 2, pad 1) * post_scale + post_shift)
        yds = conv(x, Q(wds), stride 2) * post_scale_ds + post_shift_ds
    Returns (y, yds)."""
    for t, what in ((x, "input"), (w, "weight"), (wds, "shortcut weight")):
        _require_hip_f32(t, what)
    O = ops()
    if O is None:
        raise Po2qError("po2q: qconv2d_s2ds needs the operator library (PO2Q_LIB selects another build)")
    return _op_call(O.qconv2d_s2ds, x, w, wds, int(bits), MODES[mode], int(fsr), post_scale, post_shift, ACTS[act],
                    post_scale_ds, post_shift_ds)


def conv_wgrad(x, gy, wshape, stride=1, padding=0, dilation=1, groups=1):
    """QAT backward, weight gradient of conv2d(x, w) for grad_output gy (native fp32 MFMA
    kernel, po2q_qconv2d_wgrad_f32); groups == 1 and a 1x1 / 3x3 kernel."""
    _require_hip_f32(x, "input")
    _require_hip_f32(gy, "grad_output")
    sh, sw = _pair(stride)
    ph, pw = _pair(padding)
    dh, dw = _pair(dilation)
    O = ops()
    if O is None:
        raise Po2qError("po2q: conv_wgrad needs the operator library (PO2Q_LIB selects another build)")
    return _op_call(O.conv_wgrad, x, gy, list(wshape), [sh, sw], [ph, pw], [dh, dw], int(groups))


def wgrad_supported(wshape, groups):
    """The native weight-gradient kernels cover dense 1x1 / 3x3 layers and depthwise layers
    (groups == C == K) up to 5x5."""
    K, Cg, R, S = (int(v) for v in wshape)
    if int(groups) == 1:
        return (R, S) in ((1, 1), (3, 3))
    return Cg == 1 and K == int(groups) and R * S <= 25 and S <= 5


def dilate(x, stride, size):
    """Zero insertion (po2q_dilate_f32): out[n][c][i][j] = x[n][c][i/sh][j/sw] where sh | i and
    sw | j, else 0; out is [N, C, *size].  The input gradient of a strided conv is the stride-1
    conv of dilate(dy) with the transposed, flipped weight."""
    _require_hip_f32(x, "input")
    O = ops()
    if O is None:
        raise Po2qError("po2q: dilate needs the operator library (PO2Q_LIB selects another build)")
    return _op_call(O.dilate, x, list(_pair(stride)), list(_pair(size)))


def _plan_choice(key, plan):
    """(plan index for the op, autotune flag): an explicit candidate, the PO2Q_TUNE_FILE
    record, or -1 (tuned / heuristic) with autotuning on the first call when due."""
    if plan is not None:
        return int(plan), 0
    saved = _saved_plan(key)
    if saved is not None:
        return int(saved), 0
    return -1, 1 if (key not in _tuned and _benchmark_enabled()) else 0


def _after_tune(key):
    _tuned.add(key)
    if _tune_file:
        buf = ctypes.create_string_buffer(512)
        _check(load().po2q_qconv2d_describe(*key, buf, 512))
        _save_plan(key, buf.value.decode())


def _tune_key(key):
    return ",".join(str(int(v)) for v in key)


def _load_tune_db():
    global _tune_db
    if _tune_db is None:
        _tune_db = {}
        if _tune_file and os.path.exists(_tune_file):
            import json
            with open(_tune_file) as f:
                _tune_db = json.load(f)
    return _tune_db


def _saved_plan(key):
    if not _tune_file:
        return None
    return _load_tune_db().get(_tune_key(key))


def _save_plan(key, desc):
    if not _tune_file:
        return
    import json
    L = load()
    n = L.po2q_qconv2d_plans(*key, -1, None, 0)
    buf = ctypes.create_string_buffer(512)
    for i in range(max(n, 0)):
        L.po2q_qconv2d_plans(*key, i, buf, 512)
        if buf.value.decode() == desc:
            _load_tune_db()[_tune_key(key)] = i
            with open(_tune_file, "w") as f:
                json.dump(_tune_db, f, indent=1, sort_keys=True)
            return


def _benchmark_enabled():
    on = torch.backends.cudnn.benchmark if benchmark is None else benchmark
    return bool(on) and not torch.cuda.is_current_stream_capturing()


def plans(N, C, H, W, K, R, S, stride=1, padding=0, dilation=1, groups=1, bits=4, mode="po2", fsr=1,
          precision="auto"):
    """Descriptions of the candidate plans autotuning chooses from (index 0 = heuristic default)."""
    L = load()
    sh, sw = _pair(stride)
    ph, pw = _pair(padding)
    dh, dw = _pair(dilation)
    args = (N, C, H, W, K, R, S, sh, sw, ph, pw, dh, dw, int(groups), int(bits), int(fsr), MODES[mode],
            PRECISIONS[precision])
    n = L.po2q_qconv2d_plans(*args, -1, None, 0)
    if n < 0:
        _check(-n)
    out = []
    for i in range(n):
        buf = ctypes.create_string_buffer(512)
        L.po2q_qconv2d_plans(*args, i, buf, 512)
        out.append(buf.value.decode())
    return out


def describe(N, C, H, W, K, R, S, stride=1, padding=0, dilation=1, groups=1, bits=4, mode="po2", fsr=1,
             precision="auto"):
    """The kernel plan qconv2d would run for this shape (diagnostic text)."""
    L = load()
    sh, sw = _pair(stride)
    ph, pw = _pair(padding)
    dh, dw = _pair(dilation)
    buf = ctypes.create_string_buffer(512)
    _check(L.po2q_qconv2d_describe(N, C, H, W, K, R, S, sh, sw, ph, pw, dh, dw, int(groups), int(bits), int(fsr),
                                   MODES[mode], PRECISIONS[precision], buf, 512))
    return buf.value.decode()
