"""Drop-in QuantizedConv2d (mirror of the reference's models/quantized_conv.py:5-45).

Same constructor signature and defaults (padding=1, bias=False,
quantize_fn=None, bits=4), same parameters / state_dict keys (weight[, bias]),
same get_quantization_error().  forward() runs the fused libpo2q path:

  quantize_fn in {PowerOfTwoQuantizer, PowerOfTwoPlusQuantizer}
      -> one native call: absmax + quantize + pack + conv kernels
  quantize_fn None
      -> native conv of the raw weight (reference :37-38)
  any other quantize_fn (e.g. lin / lin+ or a user Function)
      -> qw = quantize_fn.apply(weight, bits), then the native conv of qw

Backward (QAT) keeps the reference's semantics: straight-through estimator on
the weight (quantizers.py:34-36), conv gradients of the quantized weight -- the input
gradient through the native conv kernels (strided layers on zero-inserted dy), the weight
gradient through the native fp32 wgrad kernels, dense and depthwise (_QConv2dFn.backward).
HIP inputs must be fp32 (anything else raises; there is no silent fallback on the GPU).  CPU
inputs take the reference's own torch arithmetic (`_torch_forward`: the product's restated
quantizers + F.conv2d, never the oracle, never libpo2q), as the reference runs on any device.

Inference fusion: `fused(x, bn=, act=, residual=)` runs the conv
together with the eval BatchNorm that follows it in the reference's blocks (folded
into a per-channel affine), the activation and the residual add, in one native call
(po2q_qconv2d_fused_f32).  The model graphs use it when no autograd graph is being
built and the BatchNorms are in eval mode; otherwise they run the reference's module
sequence unchanged.
"""
import contextlib
import os
import threading
import weakref

import torch
import torch.nn as nn

from .. import _lib
from ..utils.quantizers import NATIVE_MODES


# False: every backward is one aten.convolution_backward of Q(w) (for A/B measurements)
NATIVE_BACKWARD = True
# backward calls that needed aten.convolution_backward for part of their gradients (tests
# assert it stays 0 on the reference models' layers)
ATEN_BACKWARD_CALLS = 0


class _QConv2dFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, stride, padding, dilation, groups, bits, mode, precision):
        y = _lib.qconv2d(x, weight, bias, stride, padding, dilation, groups, bits, mode, 1, precision)
        ctx.save_for_backward(x, weight, bias)
        ctx.conf = (stride, padding, dilation, groups, bits, mode)
        ctx.precision = precision
        return y

    @staticmethod
    def backward(ctx, gy):
        """The gradients autograd takes through F.conv2d(x, Q(w), bias) with the straight-
        through estimator on Q (quantizers.py:34-36; train.py:79-91), natively:
          input  -- the fused quantize + conv of gy (stride 1) or of gy with stride - 1 zeros
                    inserted between its pixels (po2q_dilate_f32; strided layers) with the
                    weight transposed (K <-> C within each group) and flipped, padding
                    dil * (R - 1) - pad: Q commutes with that permutation, so these are the same
                    exact PO2 weights; dense, grouped and depthwise layers alike;
          weight -- po2q_qconv2d_wgrad_f32: fp32 MFMA for dense 1x1 / 3x3 layers, a fixed-order
                    fp32 reduction for depthwise layers;
          bias   -- sum of gy over N, P, Q.
        What no kernel covers (padding beyond dil * (R - 1), grouped non-depthwise weight
        gradients, other kernel sizes) is issued as one aten.convolution_backward of Q(w)."""
        x, weight, bias = ctx.saved_tensors
        stride, padding, dilation, groups, bits, mode = ctx.conf
        gy = gy.contiguous()
        need_x, need_w = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        need_b = bias is not None and ctx.needs_input_grad[2]
        K, Cg, R, S = weight.shape
        st, pad, dil = _lib._pair(stride), _lib._pair(padding), _lib._pair(dilation)
        padl = (dil[0] * (R - 1) - pad[0], dil[1] * (S - 1) - pad[1])
        native_x = NATIVE_BACKWARD and need_x and padl[0] >= 0 and padl[1] >= 0
        native_w = NATIVE_BACKWARD and need_w and _lib.wgrad_supported(weight.shape, groups)
        gx = gw = gb = None
        if native_x:
            G = int(groups)
            wt = weight.detach().view(G, K // G, Cg, R, S).transpose(1, 2).reshape(G * Cg, K // G, R, S)
            wt = wt.flip(2, 3).contiguous()
            src = gy
            if tuple(st) != (1, 1):
                H, W = x.shape[2], x.shape[3]
                size = (H + 2 * pad[0] - dil[0] * (R - 1), W + 2 * pad[1] - dil[1] * (S - 1))
                src = _lib.dilate(gy, st, size)
            gx = _lib.qconv2d(src, wt, None, 1, padl, dil, G, bits, mode, 1, ctx.precision)
        if native_w:
            gw = _lib.conv_wgrad(x, gy, weight.shape, stride, padding, dilation, groups)
        if need_b:
            gb = gy.sum(dim=(0, 2, 3))
        rest_x, rest_w = need_x and not native_x, need_w and not native_w
        if rest_x or rest_w:
            global ATEN_BACKWARD_CALLS
            ATEN_BACKWARD_CALLS += 1
            qw = weight if mode == "none" else _lib.quantize(weight, bits, mode)
            rx, rw, _ = torch.ops.aten.convolution_backward(
                gy, x, qw, None, list(stride), list(padding), list(dilation), False, [0, 0], groups,
                [rest_x, rest_w, False])
            gx = rx if rest_x else gx
            gw = rw if rest_w else gw
        return gx, gw, gb, None, None, None, None, None, None, None


_ACT_NAMES = {nn.ReLU: "relu", nn.ReLU6: "relu6", nn.SiLU: "silu"}
_ACT_FNS = {"relu": torch.relu, "relu6": nn.functional.relu6, "silu": nn.functional.silu}


def _torch_epilogue(y, bn, act, residual):
    """bn(y) (+ residual), then the activation: the reference blocks' module order (resnet.py:64-67,
    mobilenet.py:133-134, mobile_vit.py:229-230), for the CPU path of the fused calls."""
    if bn is not None:
        y = bn(y)
    if residual is not None:
        y = y + residual
    return _ACT_FNS[act](y) if act else y


def act_name(m):
    """'relu' / 'relu6' / 'silu' for the reference's activation modules, else None."""
    return _ACT_NAMES.get(type(m))


def _fold_key(bn):
    ts = [bn.running_var, bn.running_mean] + ([bn.weight, bn.bias] if bn.affine else [])
    return (bn.eps,) + tuple((t.data_ptr(), t._version, t.device) for t in ts)


def fold_bn(bn):
    """Eval BatchNorm as (post_scale, post_shift): y = x * s + t (torch batch_norm in eval:
    (x - mean) / sqrt(var + eps) * weight + bias).

    Cached on the module, keyed on the storage and version counter of its statistics and
    affine parameters (any in-place update, load_state_dict or .to() changes the key): an eval
    forward then issues no elementwise launches for its BatchNorms (five small kernels per
    conv otherwise -- the host-side cost that made the eager fused MobileViT forward slower than
    the unfused one)."""
    key = _fold_key(bn)
    hit = getattr(bn, "_po2q_fold", None)
    if hit is not None and hit[0] == key:
        return hit[1], hit[2]
    with torch.no_grad():
        s = torch.rsqrt(bn.running_var + bn.eps)
        if bn.affine:
            s = s * bn.weight
            t = bn.bias - bn.running_mean * s
        else:
            t = -bn.running_mean * s
    bn._po2q_fold = (key, s, t)
    return s, t


# Inference fusion switch (tools/model_bench.py times both sides).
INFERENCE_FUSION = True


def can_fuse(*mods):
    """True when the inference fusion reproduces the module sequence: no autograd graph,
    every BatchNorm in eval mode with running statistics."""
    if not INFERENCE_FUSION or torch.is_grad_enabled():
        return False
    for m in mods:
        if isinstance(m, nn.modules.batchnorm._BatchNorm):
            if m.training or m.running_mean is None or m.running_var is None:
                return False
        elif m is not None and m.training:
            return False
    return True


# Batched weight staging of an eval forward (the reference quantizes each layer's weight inside
# its own forward, quantized_conv.py:35).  Layers whose kernel reads a pre-packed weight (the
# single-conv row / pointwise / depthwise plans; the pair, stride-2, chain and fused-staging
# kernels quantize their weights themselves) get their quantize + pack from ONE batched launch
# per 36 layers at the start of the forward (torch.ops.po2q.qconv2d_pack_batch), then run from
# the packed workspace (qconv2d_packed): the same plans and results, bit for bit, with every
# weight still re-quantized in every forward.  The first forward of a model at an input shape
# records which layers do that and at which shapes; later forwards at that shape pack them
# up front.  False: every layer packs its own weight (A/B runs).
BATCHED_PACKS = True
# The batched packs run inline on the forward's stream: a side stream overlapping the stem measured
# slower in the graphed model lines (config 3 521k -> 493k img/s, config 5 13.77k -> 13.47k; the fork /
# join of the second queue costs more than the ~30 us of packs it hides; profiles/r05_ab_side_packs.jsonl).
# The active forward's _ForwardPacks, per thread: concurrent eval forwards (threads, DataParallel
# replicas) each see only their own session.
_tls = threading.local()


def _session(module):
    """The calling thread's active _ForwardPacks when `module` belongs to the model that opened it."""
    sess = getattr(_tls, "packs", None)
    return sess if sess is not None and id(module) in sess.owned else None


class _ForwardPacks:
    def __init__(self, model, layers):
        self.recording = [] if layers is None else None
        self.owned = {id(m) for m in model.modules()}
        self.ws = {}
        self.fixed = {}  # id(conv) -> plan index while recording an inverted-residual block's layers
        if layers is None:
            return
        groups = {}
        for m, g, conf, plan in layers:
            groups.setdefault(conf, []).append((m, g, plan))
        for conf, items in groups.items():
            bits, mode, prec = conf
            ws = _lib.pack_batch([(m.weight, g[0], g[1], g[2], g[3], g[4]) for m, g, _ in items], bits, mode, 1,
                                 prec, plans=[pl for _, _, pl in items])
            for (m, g, pl), w in zip(items, ws):
                self.ws[id(m)] = (g, m.weight, w, pl, conf)

    def lookup(self, conv, g, weight):
        """The pack of `conv` when it was made for this geometry, this weight tensor and the layer's
        current (bits, mode, precision); None otherwise (the caller packs the layer itself)."""
        hit = self.ws.get(id(conv))
        if hit is None or hit[0] != g or hit[1] is not weight or hit[2].numel() == 0:
            return None
        if hit[4] != (conv.bits, NATIVE_MODES.get(conv.quantize_fn), conv.precision):
            return None
        return hit


# model -> {forward key: recorded layers}; weak, so a dropped model takes its records with it
_RECORDS = weakref.WeakKeyDictionary()


@contextlib.contextmanager
def batched_packs(model, x):
    """Run a model's eval forward with its single-conv layers' weight packs batched (BATCHED_PACKS)."""
    if (not BATCHED_PACKS or getattr(_tls, "packs", None) is not None or torch.is_grad_enabled() or model.training
            or not (isinstance(x, torch.Tensor) and x.is_cuda and x.dtype == torch.float32)):
        yield
        return
    # the record holds which layers read a packed weight and with which plan; it depends on the
    # layers' quantizer settings and precision as much as on the input shape
    confs = tuple((m.bits, NATIVE_MODES.get(m.quantize_fn), m.precision) for m in model.modules()
                  if isinstance(m, QuantizedConv2d))
    key = (tuple(x.shape), x.device, INFERENCE_FUSION, IR_FUSION, confs)
    rec = _RECORDS.get(model)
    if rec is None:  # keyed by the model object itself: DataParallel replicas (shallow __dict__ copies) get their own
        rec = _RECORDS[model] = {}
    sess = _ForwardPacks(model, rec.get(key))
    _tls.packs = sess
    try:
        yield
    finally:
        _tls.packs = None
    if sess.recording is not None:
        rec[key] = sess.recording


class QuantizedConv2d(nn.Conv2d):
    # conv arithmetic of the native kernels: "auto" | "fp32" | "bf16x3"
    precision = "auto"

    def __init__(
        self,
        in_channels,
        out_channels,
        kernel_size,
        stride=1,
        padding=1,
        dilation=1,
        groups=1,
        bias=False,
        quantize_fn=None,
        bits=4,
    ):
        super().__init__(in_channels, out_channels, kernel_size, stride, padding, dilation, groups, bias)
        self.quantize_fn = quantize_fn
        self.bits = bits

    def _padding(self, x):
        if isinstance(self.padding, str):
            if self.padding == "valid":
                return (0, 0)
            # 'same' (stride 1): symmetric padding when the total is even
            pads = []
            for d, k in zip(self.dilation, self.kernel_size):
                total = d * (k - 1)
                if total % 2:
                    raise RuntimeError("po2q: padding='same' with asymmetric padding is not supported")
                pads.append(total // 2)
            return tuple(pads)
        return self.padding

    def _native(self, input, weight, mode):
        if self.padding_mode != "zeros":
            raise RuntimeError("po2q: only padding_mode='zeros' is supported (the reference uses the default)")
        unbatched = input.dim() == 3
        x = input.unsqueeze(0) if unbatched else input
        y = _QConv2dFn.apply(x, weight, self.bias, self.stride, self._padding(x), self.dilation, self.groups,
                             self.bits, mode, self.precision)
        return y.squeeze(0) if unbatched else y

    def _torch_forward(self, input):
        """The reference's forward as torch ops (quantized_conv.py:32-38): F.conv2d of the quantized
        weight.  Taken for CPU tensors only -- the HIP kernels never see them -- with the product's
        own quantizers (PO2 / PO2+ via _lib.restated_quantize, lin / lin+ via
        _lib.restated_quantize_lin: the reference's torch arithmetic, bit for bit on CPU)."""
        if self.quantize_fn is None:
            return self._conv_forward(input, self.weight, self.bias)
        return self._conv_forward(input, self.quantize_fn.apply(self.weight, self.bits), self.bias)

    def forward(self, input):
        # reference quantized_conv.py:32-38
        if not input.is_cuda:
            return self._torch_forward(input)
        if self.quantize_fn is None:
            return self._native(input, self.weight, "none")
        mode = NATIVE_MODES.get(self.quantize_fn)
        if mode is not None:
            return self._native(input, self.weight, mode)
        quantized_weight = self.quantize_fn.apply(self.weight, self.bits)
        return self._native(input, quantized_weight, "none")

    def fused(self, input, bn=None, act=None, residual=None):
        """act(bn(self(input)) + residual) in one native call (eval, no autograd; see
        can_fuse).  bn: the following eval BatchNorm or None; act: None | 'relu' |
        'relu6' | 'silu'."""
        if not input.is_cuda:  # CPU: the reference's module sequence (conv -> bn -> + residual -> act)
            return _torch_epilogue(self(input), bn, act, residual)
        if self.padding_mode != "zeros":
            raise RuntimeError("po2q: only padding_mode='zeros' is supported (the reference uses the default)")
        mode = "none" if self.quantize_fn is None else NATIVE_MODES.get(self.quantize_fn)
        weight = self.weight
        if mode is None:  # a non-native quantizer (lin / lin+ / user Function): quantize first
            weight = self.quantize_fn.apply(self.weight, self.bits)
            mode = "none"
        ps, pb = fold_bn(bn) if bn is not None else (None, None)
        sess = _session(self)
        if sess is not None and mode != "none" and input.dim() == 4:
            g = (tuple(input.shape), tuple(self.stride), tuple(self._padding(input)), tuple(self.dilation), self.groups)
            if sess.recording is not None:
                sess.recording.append((self, g, (self.bits, mode, self.precision), sess.fixed.get(id(self))))
            else:
                hit = sess.lookup(self, g, weight)
                if hit is not None:
                    return _lib.qconv2d_packed(input, weight, hit[2], self.bias, g[1], g[2], g[3], g[4], self.bits,
                                               mode, 1, self.precision, post_scale=ps, post_shift=pb,
                                               residual=residual, act=act or "none", plan=hit[3])
        return _lib.qconv2d_fused(input, weight, self.bias, self.stride, self._padding(input), self.dilation,
                                  self.groups, self.bits, mode, 1, self.precision, post_scale=ps, post_shift=pb,
                                  residual=residual, act=act or "none")

    def get_quantization_error(self):
        # reference quantized_conv.py:40-45
        if self.quantize_fn is not None:
            quantized_weight = self.quantize_fn.apply(self.weight, self.bits)
            return torch.sum((quantized_weight - self.weight) ** 2), self.weight.numel()
        else:
            return 0, self.weight.numel()



def plain_conv(conv, x):
    """An unquantized nn.Conv2d (the reference's stems: resnet.py:99-102) on a HIP fp32 input through
    the native fp32 kernels with the native backward (_QConv2dFn, mode "none": exact fp32 products,
    the weight gradient from the fixed-order wgrad kernels, so a training step is deterministic run to
    run); any other input runs the module itself."""
    if (not (x.is_cuda and x.dtype == torch.float32 and x.dim() == 4) or conv.padding_mode != "zeros"
            or isinstance(conv.padding, str)):
        return conv(x)
    return _QConv2dFn.apply(x, conv.weight, conv.bias, conv.stride, conv.padding, conv.dilation, conv.groups, 4,
                            "none", "auto")


def plain_conv_fused(conv, x, bn=None, act=None, residual=None):
    """An unquantized nn.Conv2d (the reference's stems and last 1x1 convs: resnet.py:99-102,
    mobilenet.py:41-50, mobile_vit.py:41-48) with the eval BatchNorm / activation after it, as
    ONE native call of the fp32 path (mode "none": exact fp32 products, fp32 accumulation)."""
    if not x.is_cuda:
        return _torch_epilogue(conv(x), bn, act, residual)
    if conv.padding_mode != "zeros" or isinstance(conv.padding, str):
        raise RuntimeError("po2q: fused plain conv needs numeric zero padding")
    ps, pb = fold_bn(bn) if bn is not None else (None, None)
    return _lib.qconv2d_fused(x, conv.weight, conv.bias, conv.stride, conv.padding, conv.dilation, conv.groups, 4,
                              "none", 1, "auto", post_scale=ps, post_shift=pb, residual=residual, act=act or "none")


def _native_ok(x):
    return x.is_cuda and x.dtype == torch.float32 and x.dim() == 4


def fusable_sequence(seq):
    """True when seq is (conv, BatchNorm[, activation])* -- the conv blocks of the reference's
    models (mobilenet.py:53-131, mobile_vit.py:15-48, 131-233); conv is a QuantizedConv2d or an
    unquantized nn.Conv2d with numeric zero padding."""
    mods = list(seq)
    i = 0
    while i < len(mods):
        c = mods[i]
        if not isinstance(c, nn.Conv2d) or c.padding_mode != "zeros" or isinstance(c.padding, str):
            return False
        i += 1
        if i < len(mods) and isinstance(mods[i], nn.modules.batchnorm._BatchNorm):
            i += 1
        if i < len(mods) and act_name(mods[i]) is not None:
            i += 1
    return True


def run_fused_sequence(seq, x, residual=None):
    """seq(x) (+ residual) with every (conv, BN, activation) group as one fused native
    call; the residual is added by the last group, after its BN and before its
    activation (the reference adds it after a BN-terminated group: mobilenet.py:133-134,
    mobile_vit.py:229-230)."""
    mods = list(seq)
    i = 0
    while i < len(mods):
        conv = mods[i]
        i += 1
        bn = None
        if i < len(mods) and isinstance(mods[i], nn.modules.batchnorm._BatchNorm):
            bn = mods[i]
            i += 1
        act = act_name(mods[i]) if i < len(mods) else None
        if act is not None:
            i += 1
        res = residual if i >= len(mods) else None
        if isinstance(conv, QuantizedConv2d):
            x = conv.fused(x, bn=bn, act=act, residual=res)
        else:
            x = plain_conv_fused(conv, x, bn=bn, act=act, residual=res)
    return x


# Whole inverted-residual blocks (mobilenet.py:53-134, mobile_vit.py:131-239) as ONE launch
# (torch.ops.po2q.qconv2d_ir: expand -> depthwise -> project with the hidden activations on
# chip) inside a batched_packs forward, from the three layers' batched packs.  The op fuses only
# where the block kernel measured faster than the three fused layer launches replayed from a HIP
# graph -- the small-image kernel at 3x3 / 4x4 (po2q_qconv2d_ir_supported; profiles/r04_ir_ab.jsonl,
# r04_ir_small_ab.jsonl) -- and runs the layers from the same packs elsewhere.  False: always the
# layer calls (A/B runs).
IR_FUSION = True


def _ir_spec(seq):
    """(expand | None, depthwise, project) (conv, bn, act) groups when seq is an inverted-residual
    conv block the fused kernel reproduces: bias-free QuantizedConv2d layers with one native
    quantizer / bits / precision, 1x1 expand, 3x3 pad-1 depthwise (stride 1 or 2), 1x1 project."""
    spec = seq.__dict__.get("_po2q_ir")
    if spec is not None:
        return spec or None
    groups, mods, i = [], list(seq), 0
    while i < len(mods):
        conv, bn, act = mods[i], None, None
        i += 1
        if i < len(mods) and isinstance(mods[i], nn.modules.batchnorm._BatchNorm):
            bn, i = mods[i], i + 1
        if i < len(mods) and act_name(mods[i]) is not None:
            act, i = act_name(mods[i]), i + 1
        groups.append((conv, bn, act))
    ok = len(groups) in (2, 3) and all(isinstance(g[0], QuantizedConv2d) for g in groups)
    if ok:
        convs = [g[0] for g in groups]
        conf = {(c.bits, c.quantize_fn, c.precision) for c in convs}
        ok = (len(conf) == 1 and NATIVE_MODES.get(convs[0].quantize_fn) is not None
              and all(c.bias is None and c.padding_mode == "zeros" and not isinstance(c.padding, str)
                      and tuple(c.dilation) == (1, 1) for c in convs))
    if ok:
        d, p = convs[-2], convs[-1]
        pw = lambda c: tuple(c.kernel_size) == (1, 1) and tuple(c.stride) == (1, 1) and tuple(c.padding) == (0, 0) \
            and c.groups == 1
        ok = (tuple(d.kernel_size) == (3, 3) and tuple(d.padding) == (1, 1) and d.stride[0] == d.stride[1]
              and d.stride[0] in (1, 2) and d.groups == d.in_channels == d.out_channels and pw(p)
              and (len(convs) == 2 or pw(convs[0])))
    spec = (([None] if len(groups) == 2 else []) + groups) if ok else ()
    seq.__dict__["_po2q_ir"] = spec
    return spec or None


def run_inverted_residual(seq, x, residual=None):
    """run_fused_sequence(seq, x, residual) for an inverted-residual conv block: ONE qconv2d_ir launch
    when a batched_packs forward holds the three layers' packs, else the per-layer fused calls
    (which record the layers for the next forward's packs)."""
    sess = _session(seq)
    spec = _ir_spec(seq) if IR_FUSION and sess is not None else None
    if spec is not None and x.dim() == 4:  # only blocks the kernel takes: the others keep their tuned plans
        d = spec[1][0]
        if not _lib.ir_shape_supported(x.shape, d.out_channels, spec[2][0].out_channels, d.stride[0],
                                       spec[0] is not None):
            spec = None
    if spec is not None and sess.recording is not None:
        # record the block's layers with their heuristic plans (candidate 0: the pointwise and
        # depthwise kernels whose packs the block kernel reads), whatever the autotuner picked
        for g in spec:
            if g is not None:
                sess.fixed[id(g[0])] = 0
        spec = None
    if spec is not None and x.dim() == 4:
        hits = []
        for g in spec:
            hit = sess.ws.get(id(g[0])) if g is not None else None
            if g is not None:
                hit = sess.lookup(g[0], hit[0], g[0].weight) if hit is not None else None
                if hit is None or hit[3] != 0:
                    break
            hits.append(hit)
        else:
            e, d, p = spec
            if (hits[0] if e is not None else hits[1])[0][0] == tuple(x.shape):
                f = [fold_bn(g[1]) if g is not None and g[1] is not None else (None, None) for g in spec]
                conv = d[0]
                return _lib.qconv2d_ir(x, e[0].weight if e else None, d[0].weight, p[0].weight,
                                       hits[0][2] if e else None, hits[1][2], hits[2][2], conv.stride[0], conv.bits,
                                       NATIVE_MODES[conv.quantize_fn], 1, conv.precision,
                                       f[0][0], f[0][1], e[2] if e else None, f[1][0], f[1][1], d[2], f[2][0],
                                       f[2][1], residual, p[2])
    return run_fused_sequence(seq, x, residual=residual)


def run_sequence(seq, x):
    """seq(x): the fused native calls in eval (can_fuse) when seq is a fusable conv block and x a
    HIP fp32 tensor, else the module sequence itself."""
    if _native_ok(x) and can_fuse(*seq) and fusable_sequence(seq):
        return run_fused_sequence(seq, x)
    return seq(x)
