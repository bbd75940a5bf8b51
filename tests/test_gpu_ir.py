"""GPU parity of the fused inverted-residual block (po2q_qconv2d_ir_f32 / torch.ops.po2q.qconv2d_ir):
expand 1x1 -> BN -> act -> depthwise 3x3 -> BN -> act -> project 1x1 -> BN (+ x) (reference
models/mobilenet.py:53-134, MobileViT's MV2Block models/mobile_vit.py:131-239; every conv a
QuantizedConv2d.forward, models/quantized_conv.py:32-38) in one launch, against the oracle (C
restatement of the reference quantizer + fp64 direct conv, oracle/), against the same chain in
torch fp32 on Q(w) and against the three single-layer calls from the same packs.  Bar: normwise
1e-5 (CONV_TOL)."""
import ctypes

import numpy as np

import pytest
import torch
import torch.nn.functional as F

from po2_quantization_amd import _lib
from po2_quantization_amd.models import quantized_conv as qc
from po2_quantization_amd.models.model import get_model
from po2_quantization_amd.utils.quantizers import quantizer_dict
from tests._util import CONV_TOL

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
ACT = {"none": lambda t: t, "relu": torch.relu, "relu6": F.relu6, "silu": F.silu}


def nerr(y, ref):
    return ((y - ref).abs().max() / ref.abs().max()).item()


def make_block(N, Cin, Ch, Cout, H, W, seed, expand=True):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(N, Cin, H, W, generator=g)
    we = torch.randn(Ch, Cin, 1, 1, generator=g) * (1.0 / Cin ** 0.5) if expand else None
    wd = torch.randn(Ch, 1, 3, 3, generator=g) * 0.3
    wp = torch.randn(Cout, Ch, 1, 1, generator=g) * (1.0 / Ch ** 0.5)
    bn = [((torch.rand(c, generator=g) + 0.5), torch.randn(c, generator=g) * 0.1) for c in (Ch, Ch, Cout)]
    to = lambda t: None if t is None else t.to(DEV)
    return to(x), to(we), to(wd), to(wp), [(to(s), to(b)) for s, b in bn]


def torch_block(x, we, wd, wp, bn, stride, acts, residual, mode, bits):
    h = x
    if we is not None:
        h = F.conv2d(x, _lib.quantize(we, bits, mode))
        h = ACT[acts[0]](h * bn[0][0].view(1, -1, 1, 1) + bn[0][1].view(1, -1, 1, 1))
    d = F.conv2d(h, _lib.quantize(wd, bits, mode), None, stride, 1, 1, wd.shape[0])
    d = ACT[acts[1]](d * bn[1][0].view(1, -1, 1, 1) + bn[1][1].view(1, -1, 1, 1))
    y = F.conv2d(d, _lib.quantize(wp, bits, mode))
    y = y * bn[2][0].view(1, -1, 1, 1) + bn[2][1].view(1, -1, 1, 1)
    if residual is not None:
        y = y + residual
    return ACT[acts[2]](y)


def oracle_ir_block(x, we, wd, wp, bn, stride, acts, residual, mode, bits):
    """The reference's inverted-residual block (mobilenet.py:89-134; MV2Block mobile_vit.py:131-239) on
    the oracle: O.qconv2d (fp64 accumulation on the bit-exact Q(w), oracle/po2_oracle.c) for every
    conv, the eval BatchNorm as its per-channel affine and the activation in numpy, each intermediate
    rounded to fp32 as the reference's tensors are.  Test-only checker."""
    from oracle import oracle as O

    acts_np = {"none": lambda t: t, "relu": lambda t: np.maximum(t, 0.0), "relu6": lambda t: np.clip(t, 0.0, 6.0),
               "silu": lambda t: t / (1.0 + np.exp(-t))}
    v = lambda t: t.cpu().numpy().astype(np.float64).reshape(1, -1, 1, 1)  # noqa: E731
    h = x.cpu().numpy()
    if we is not None:
        c, _ = O.qconv2d(h, we.cpu().numpy(), None, 1, 0, 1, 1, bits, mode)
        h = acts_np[acts[0]](c.astype(np.float32) * v(bn[0][0]) + v(bn[0][1])).astype(np.float32)
    Ch = wd.shape[0]
    d, _ = O.qconv2d(h, wd.cpu().numpy(), None, stride, 1, 1, Ch, bits, mode)
    d = acts_np[acts[1]](d.astype(np.float32) * v(bn[1][0]) + v(bn[1][1])).astype(np.float32)
    y, _ = O.qconv2d(d, wp.cpu().numpy(), None, 1, 0, 1, 1, bits, mode)
    y = y.astype(np.float32) * v(bn[2][0]) + v(bn[2][1])
    if residual is not None:
        y = y + residual.cpu().numpy().astype(np.float64)
    return acts_np[acts[2]](y)


def packs(x, we, wd, wp, stride, bits, mode):
    N, Cin, H, W = x.shape
    Ch = wd.shape[0]
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    layers = ([(we, x.shape, 1, 0, 1, 1)] if we is not None else []) + [
        (wd, (N, Ch, H, W), stride, 1, 1, Ch), (wp, (N, Ch, Ho, Wo), 1, 0, 1, 1)]
    ws = _lib.pack_batch(layers, bits, mode)
    return ([ws[0]] if we is not None else [None]) + ws[-2:]


def run_ir(x, we, wd, wp, bn, stride, acts, residual, mode, bits):
    ws_e, ws_d, ws_p = packs(x, we, wd, wp, stride, bits, mode)
    return _lib.qconv2d_ir(x, we, wd, wp, ws_e, ws_d, ws_p, stride, bits, mode, ps1=bn[0][0], pb1=bn[0][1],
                           act1=acts[0], ps2=bn[1][0], pb2=bn[1][1], act2=acts[1], ps3=bn[2][0], pb3=bn[2][1],
                           residual=residual, act3=acts[2])


def layer_chain(x, we, wd, wp, bn, stride, acts, residual, mode, bits):
    ws_e, ws_d, ws_p = packs(x, we, wd, wp, stride, bits, mode)
    h = x
    if we is not None:
        h = _lib.qconv2d_packed(x, we, ws_e, None, 1, 0, 1, 1, bits, mode, post_scale=bn[0][0], post_shift=bn[0][1],
                                act=acts[0])
    d = _lib.qconv2d_packed(h, wd, ws_d, None, stride, 1, 1, wd.shape[0], bits, mode, post_scale=bn[1][0],
                            post_shift=bn[1][1], act=acts[1])
    return _lib.qconv2d_packed(d, wp, ws_p, None, 1, 0, 1, 1, bits, mode, post_scale=bn[2][0], post_shift=bn[2][1],
                               residual=residual, act=acts[2])


# (N, Cin, Ch, Cout, H, W, stride, expand): every MobileNetV2 block at 32x32 input (the stem is
# stride 2: 16x16 .. 1x1), ImageNet-size bands (112 / 56 / 28), ragged and odd shapes (hidden
# width with a 16-channel tail chunk, G-image groups with a partial last group, non-square).
SHAPES = [(3, 32, 32, 16, 16, 16, 1, False), (3, 16, 96, 24, 16, 16, 2, True), (3, 24, 144, 24, 8, 8, 1, True),
          (3, 24, 144, 32, 8, 8, 2, True), (3, 32, 192, 32, 4, 4, 1, True), (3, 32, 192, 64, 4, 4, 2, True),
          (3, 64, 384, 64, 2, 2, 1, True), (3, 64, 384, 96, 2, 2, 1, True), (3, 96, 576, 96, 2, 2, 1, True),
          (3, 96, 576, 160, 2, 2, 2, True), (3, 160, 960, 160, 1, 1, 1, True), (3, 160, 960, 320, 1, 1, 1, True),
          (1, 16, 96, 24, 112, 112, 2, True), (2, 24, 144, 24, 56, 56, 1, True), (2, 32, 192, 32, 28, 28, 1, True),
          (1, 32, 32, 16, 112, 112, 1, False), (5, 8, 48, 8, 7, 7, 1, True), (37, 16, 64, 16, 3, 3, 1, True),
          (1025, 16, 32, 24, 2, 2, 1, True), (1031, 8, 32, 8, 1, 1, 1, True), (2, 12, 80, 20, 9, 13, 2, True),
          (2, 20, 40, 20, 11, 6, 1, True)]


# kernel selection: "default" = the small-image kernel for 3x3 / 4x4 images, the layer launches
# elsewhere; "small" = the small-image kernel for every image <= 16 pixels; "chunked" = the chunked
# kernel for every shape (opt-in knobs)
KERNELS = {"default": {}, "small": {"PO2Q_IR_SMALL": "1"}, "chunked": {"PO2Q_IR_LARGE": "1", "PO2Q_IR_SMALL": "0"}}


@pytest.mark.parametrize("shape", SHAPES, ids=[str(s) for s in SHAPES])
@pytest.mark.parametrize("mode,bits", [("po2", 4), ("po2+", 3)])
@pytest.mark.parametrize("kernel", list(KERNELS))
def test_ir_block_vs_torch_and_layers(shape, mode, bits, kernel, monkeypatch):
    for k, v in KERNELS[kernel].items():
        monkeypatch.setenv(k, v)
    N, Cin, Ch, Cout, H, W, s, expand = shape
    x, we, wd, wp, bn = make_block(N, Cin, Ch, Cout, H, W, hash(shape) & 0xFFFF, expand)
    res = x if (s == 1 and Cin == Cout) else None
    acts = ("relu6", "relu6", "none")
    y = run_ir(x, we, wd, wp, bn, s, acts, res, mode, bits)
    ref = torch_block(x, we, wd, wp, bn, s, acts, res, mode, bits)
    assert y.shape == ref.shape
    assert nerr(y, ref) <= CONV_TOL, nerr(y, ref)
    lay = layer_chain(x, we, wd, wp, bn, s, acts, res, mode, bits)
    assert nerr(y, lay) <= CONV_TOL, nerr(y, lay)


@pytest.mark.parametrize("shape", SHAPES, ids=[str(s) for s in SHAPES])
@pytest.mark.parametrize("mode,bits", [("po2", 4), ("po2+", 3)])
@pytest.mark.parametrize("kernel", list(KERNELS))
def test_ir_block_vs_oracle(shape, mode, bits, kernel, monkeypatch):
    """Every SHAPES block through every kernel selection against the oracle block."""
    from tests._util import normwise_err

    for k, v in KERNELS[kernel].items():
        monkeypatch.setenv(k, v)
    N, Cin, Ch, Cout, H, W, s, expand = shape
    x, we, wd, wp, bn = make_block(N, Cin, Ch, Cout, H, W, (hash(shape) + 17) & 0xFFFF, expand)
    res = x if (s == 1 and Cin == Cout) else None
    acts = ("relu6", "relu6", "none")
    y = run_ir(x, we, wd, wp, bn, s, acts, res, mode, bits).cpu().numpy()
    ref = oracle_ir_block(x, we, wd, wp, bn, s, acts, res, mode, bits)
    assert y.shape == ref.shape
    assert normwise_err(y, ref) <= CONV_TOL, normwise_err(y, ref)


@pytest.mark.parametrize("acts", [("silu", "silu", "none"), ("relu", "relu6", "relu"), ("none", "none", "silu")])
@pytest.mark.parametrize("hw", [8, 2])
def test_ir_block_activations(acts, hw, monkeypatch):
    """MobileViT's MV2Block uses SiLU (mobile_vit.py:131-239); every activation at every position,
    in the chunked (8x8) and the small-image (2x2) kernel, against torch and the oracle."""
    from tests._util import normwise_err

    monkeypatch.setenv("PO2Q_IR_LARGE", "1")
    x, we, wd, wp, bn = make_block(4, 16, 64, 16, hw, hw, 7)
    y = run_ir(x, we, wd, wp, bn, 1, acts, x, "po2+", 4)
    ref = torch_block(x, we, wd, wp, bn, 1, acts, x, "po2+", 4)
    assert nerr(y, ref) <= CONV_TOL, nerr(y, ref)
    oref = oracle_ir_block(x, we, wd, wp, bn, 1, acts, x, "po2+", 4)
    assert normwise_err(y.cpu().numpy(), oref) <= CONV_TOL, normwise_err(y.cpu().numpy(), oref)


@pytest.mark.parametrize("shape", [(40, 64, 384, 96, 2, 2, 1), (33, 160, 960, 320, 1, 1, 1), (17, 32, 192, 64, 4, 4, 2),
                                   (9, 24, 96, 24, 3, 3, 1), (5, 96, 576, 160, 2, 2, 2), (3, 16, 64, 200, 1, 1, 1)],
                         ids=str)
def test_ir_small_kernel_groups(shape, monkeypatch):
    """The small-image kernel: G images per block (16 at 1x1, 4 at 2x2, 1 from 3x3; below 3x3 opt-in),
    partial last groups, two output-tile wave groups (Cout > 192), stride 2, a 3x3 image (9 of 16 tile
    rows)."""
    monkeypatch.setenv("PO2Q_IR_SMALL", "1")
    N, Cin, Ch, Cout, H, W, s = shape
    x, we, wd, wp, bn = make_block(N, Cin, Ch, Cout, H, W, N + Ch)
    res = x if (s == 1 and Cin == Cout) else None
    acts = ("relu6", "relu6", "none")
    y = run_ir(x, we, wd, wp, bn, s, acts, res, "po2", 4)
    ref = torch_block(x, we, wd, wp, bn, s, acts, res, "po2", 4)
    assert nerr(y, ref) <= CONV_TOL, nerr(y, ref)
    lay = layer_chain(x, we, wd, wp, bn, s, acts, res, "po2", 4)
    assert nerr(y, lay) <= CONV_TOL, nerr(y, lay)


def test_ir_unsupported_shape_runs_the_layers():
    """A hidden width that is not a multiple of 16 has no block geometry: the op runs the three
    layers from the same packs (the same HIP kernels), and the result is still the chain."""
    x, we, wd, wp, bn = make_block(2, 5, 30, 7, 6, 6, 3)
    acts = ("relu6", "relu6", "none")
    y = run_ir(x, we, wd, wp, bn, 1, acts, None, "po2", 4)
    ref = torch_block(x, we, wd, wp, bn, 1, acts, None, "po2", 4)
    assert nerr(y, ref) <= CONV_TOL


def test_ir_rejects_bad_arguments():
    x, we, wd, wp, bn = make_block(2, 16, 32, 16, 4, 4, 1)
    ws_e, ws_d, ws_p = packs(x, we, wd, wp, 1, 4, "po2")
    with pytest.raises(_lib.Po2qError, match="expand weight"):
        _lib.qconv2d_ir(x, we[:, :8], wd, wp, ws_e, ws_d, ws_p, 1, 4, "po2")
    with pytest.raises(_lib.Po2qError, match="stride"):
        _lib.qconv2d_ir(x, we, wd, wp, ws_e, ws_d, ws_p, 3, 4, "po2")
    with pytest.raises(_lib.Po2qError, match="residual"):
        _lib.qconv2d_ir(x, we, wd, wp, ws_e, ws_d, ws_p, 1, 4, "po2", residual=x[:, :8])
    with pytest.raises(_lib.Po2qError, match="ps1"):
        _lib.qconv2d_ir(x, we, wd, wp, ws_e, ws_d, ws_p, 1, 4, "po2", ps1=bn[2][0][:3])


def _plan(L, N, C, H, W, K, R, S, st, pad, groups, bits, mode):
    h = ctypes.c_void_p()
    assert L.po2q_qconv2d_plan_create(ctypes.byref(h), -1, N, C, H, W, K, R, S, st, st, pad, pad, 1, 1, groups, bits,
                                      1, _lib.MODES[mode], 0) == 0, L.po2q_last_error()
    return h


def test_ir_through_the_c_abi(monkeypatch):
    """The C ABI as a non-torch binding uses it: plan handles, po2q_qconv2d_plan_pack_batch, then
    po2q_qconv2d_ir_supported / po2q_qconv2d_ir_f32 on the current stream (8x8: the chunked kernel,
    opt-in)."""
    monkeypatch.setenv("PO2Q_IR_LARGE", "1")
    L = _lib.load()
    N, Cin, Ch, Cout, H, s = 4, 24, 144, 24, 8, 1
    x, we, wd, wp, bn = make_block(N, Cin, Ch, Cout, H, H, 21)
    hs = [_plan(L, N, Cin, H, H, Ch, 1, 1, 1, 0, 1, 4, "po2"), _plan(L, N, Ch, H, H, Ch, 3, 3, s, 1, Ch, 4, "po2"),
          _plan(L, N, Ch, H, H, Cout, 1, 1, 1, 0, 1, 4, "po2")]
    try:
        assert L.po2q_qconv2d_ir_supported(hs[0], hs[1], hs[2]) == 1, L.po2q_last_error()
        assert L.po2q_qconv2d_ir_supported(hs[2], hs[1], hs[0]) == 0  # not a chain
        nb = [L.po2q_qconv2d_plan_workspace_bytes(h) for h in hs]
        wss = [torch.empty(b, dtype=torch.uint8, device=DEV) for b in nb]
        P = ctypes.c_void_p
        st = L.po2q_qconv2d_plan_pack_batch(3, (P * 3)(*[h.value for h in hs]),
                                            (P * 3)(*[t.data_ptr() for t in (we, wd, wp)]),
                                            (P * 3)(*[t.data_ptr() for t in wss]), (ctypes.c_size_t * 3)(*nb),
                                            _lib._stream(x.device))
        assert st == 0, L.po2q_last_error()
        y = torch.empty(N, Cout, H, H, device=DEV)
        ptr = lambda t: t.data_ptr()
        st = L.po2q_qconv2d_ir_f32(ptr(x), ptr(y), hs[0], ptr(wss[0]), nb[0], hs[1], ptr(wss[1]), nb[1], hs[2],
                                   ptr(wss[2]), nb[2], ptr(bn[0][0]), ptr(bn[0][1]), 2, ptr(bn[1][0]), ptr(bn[1][1]), 2,
                                   ptr(bn[2][0]), ptr(bn[2][1]), ptr(x), 0, _lib._stream(x.device))
        assert st == 0, L.po2q_last_error()
        torch.cuda.synchronize()
        ref = torch_block(x, we, wd, wp, bn, s, ("relu6", "relu6", "none"), x, "po2", 4)
        assert nerr(y, ref) <= CONV_TOL, nerr(y, ref)
        st = L.po2q_qconv2d_ir_f32(ptr(x), ptr(y), hs[0], ptr(wss[0]), 16, hs[1], ptr(wss[1]), nb[1], hs[2],
                                   ptr(wss[2]), nb[2], None, None, 0, None, None, 0, None, None, None, 0,
                                   _lib._stream(x.device))
        assert st == 3 and b"workspace" in L.po2q_last_error()
    finally:
        for h in hs:
            L.po2q_qconv2d_plan_destroy(h)


@pytest.mark.parametrize("name,image,q,bits", [("mobilenet", 32, "po2+", 4), ("mobilenet", 64, "po2", 4),
                                               ("mobilevit", 64, "po2+", 2)])
def test_model_forward_ir_fusion(name, image, q, bits, monkeypatch):
    """Eval forwards with the blocks as one launch each (IR_FUSION, the default) equal the per-layer
    forwards at the 1e-5 bar (normwise)."""
    torch.manual_seed(0)
    m = get_model(name, 10, quantizer_dict[q], bits, (image, image)).to(DEV).eval()
    for mod in m.modules():  # non-trivial BN statistics
        if isinstance(mod, torch.nn.BatchNorm2d):
            mod.running_mean.uniform_(-0.1, 0.1)
            mod.running_var.uniform_(0.5, 1.5)
    x = torch.randn(6, 3, image, image, device=DEV)
    calls = []
    real = _lib.qconv2d_ir
    monkeypatch.setattr(_lib, "qconv2d_ir", lambda *a, **k: calls.append(1) or real(*a, **k))
    with torch.no_grad():
        monkeypatch.setattr(qc, "IR_FUSION", False)  # every block as its three layer calls
        ref = m(x)
        ref2 = m(x)
        monkeypatch.setattr(qc, "IR_FUSION", True)
        m(x)  # the recording forward of this shape happened above
        y = m(x)
    assert calls, "the fused block op never ran"
    assert torch.equal(ref, ref2)
    assert nerr(y, ref) <= CONV_TOL, nerr(y, ref)
