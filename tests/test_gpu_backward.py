"""GPU parity of the native QAT backward: the gradients autograd takes
through F.conv2d(x, Q(w), bias) with the straight-through estimator on Q (reference
utils/quantizers.py:34-36, train.py:79-91), against torch's own convolution_backward of
the bit-exact Q(w) in fp64 on the CPU (a plain PyTorch reference).  Bar: normwise 1e-5."""
import pytest
import torch

from po2_quantization_amd import _lib
from po2_quantization_amd.models.quantized_conv import QuantizedConv2d
from po2_quantization_amd.utils.quantizers import quantizer_dict
from tests._util import CONV_TOL

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def nerr(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-300))


def ref_grads(x, w, b, gy, qn, bits, stride, pad, groups=1, dil=1):
    qw = w if qn is None else _lib.quantize(w, bits, qn)
    gx, gw, gb = torch.ops.aten.convolution_backward(
        gy.double().cpu(), x.double().cpu(), qw.double().cpu(), None if b is None else [b.shape[0]],
        [stride, stride], [pad, pad], [dil, dil], False, [0, 0], groups, [True, True, b is not None])
    return gx, gw, gb


SHAPES = [  # N, C, H, W, K, R, stride, pad, bias, quantizer
    (2, 16, 20, 20, 16, 3, 1, 1, False, "po2"),
    (2, 32, 12, 12, 32, 3, 1, 1, False, "po2+"),
    (1, 64, 10, 10, 64, 3, 1, 1, True, "po2"),
    (2, 16, 17, 17, 32, 3, 2, 1, False, "po2"),    # stride 2: input grad on zero-inserted dy
    (2, 16, 16, 16, 32, 1, 2, 0, False, "po2+"),   # 1x1 projection
    (1, 8, 9, 70, 24, 3, 1, 1, True, "po2"),       # ragged channels / columns
    (3, 16, 8, 8, 16, 3, 1, 1, False, None),       # plain conv (quantize_fn None)
    (2, 20, 7, 5, 36, 3, 1, 2, False, "po2"),      # padding 2 (input grad padding 0)
]


@pytest.mark.parametrize("shape", SHAPES, ids=[str(s) for s in SHAPES])
def test_qconv_backward_vs_torch_fp64(shape):
    N, C, H, W, K, R, st, pad, bias, qn = shape
    g = torch.Generator().manual_seed(N * 1000 + C * 10 + K)
    conv = QuantizedConv2d(C, K, R, stride=st, padding=pad, bias=bias,
                           quantize_fn=quantizer_dict[qn] if qn else None, bits=4)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(conv.weight.shape, generator=g) * 0.2)
        if bias:
            conv.bias.copy_(torch.randn(K, generator=g))
    conv = conv.to(DEV)
    x = torch.randn(N, C, H, W, generator=g).to(DEV).requires_grad_(True)
    y = conv(x)
    gy = torch.randn(y.shape, generator=g).to(DEV)
    y.backward(gy)
    rx, rw, rb = ref_grads(x.detach(), conv.weight.detach(), conv.bias, gy, qn, 4, st, pad)
    assert nerr(x.grad, rx) <= CONV_TOL, nerr(x.grad, rx)
    assert nerr(conv.weight.grad, rw) <= CONV_TOL, nerr(conv.weight.grad, rw)
    if bias:
        assert nerr(conv.bias.grad, rb) <= CONV_TOL


@pytest.mark.parametrize("layer", [(16, 224, 16, 3, 1, 1), (32, 112, 32, 3, 1, 1), (64, 56, 64, 3, 1, 1),
                                   (16, 224, 32, 3, 2, 1), (32, 112, 64, 1, 2, 0)])
def test_full_size_resnet56_backward_vs_torch(layer):
    """ResNet56 @224 layer shapes (bs = 16): native input / weight gradients against
    torch's fp32 GPU convolution_backward of Q(w)."""
    C, H, K, R, st, pad = layer
    torch.manual_seed(3)
    x = torch.relu(torch.randn(16, C, H, H, device=DEV))
    w = torch.randn(K, C, R, R, device=DEV) * (2.0 / (K * R * R)) ** 0.5
    P = (H + 2 * pad - R) // st + 1
    gy = torch.randn(16, K, P, P, device=DEV)
    gw = _lib.conv_wgrad(x, gy, w.shape, st, pad, 1, 1)
    qw = _lib.quantize(w, 4, "po2")
    rx, rw, _ = torch.ops.aten.convolution_backward(gy, x, qw, None, [st, st], [pad, pad], [1, 1], False, [0, 0], 1,
                                                     [True, True, False])
    assert nerr(gw, rw) <= CONV_TOL, nerr(gw, rw)
    if st == 1:
        wt = w.flip(2, 3).transpose(0, 1).contiguous()
        gx = _lib.qconv2d(gy, wt, None, 1, R - 1 - pad, 1, 1, 4, "po2")
        assert nerr(gx, rx) <= CONV_TOL, nerr(gx, rx)


def test_wgrad_deterministic_and_unsupported():
    torch.manual_seed(4)
    x = torch.randn(4, 32, 24, 24, device=DEV)
    gy = torch.randn(4, 16, 24, 24, device=DEV)
    a = _lib.conv_wgrad(x, gy, (16, 32, 3, 3), 1, 1)
    b = _lib.conv_wgrad(x, gy, (16, 32, 3, 3), 1, 1)
    assert torch.equal(a, b)  # fixed summation order, no atomics
    assert not _lib.wgrad_supported((16, 32, 5, 5), 1) and not _lib.wgrad_supported((16, 8, 3, 3), 4)
    with pytest.raises(_lib.Po2qError):
        _lib.conv_wgrad(x, gy, (16, 32, 5, 5), 1, 2)


def test_wgrad_rejects_mismatched_shapes():
    """The C ABI takes no grad_output / gradient shapes, so the op checks them: a weight whose
    input channels differ from x's, or a grad_output that is not [N, K, P, Q], raises instead of
    reading or writing out of bounds."""
    x = torch.randn(2, 32, 12, 12, device=DEV)
    gy = torch.randn(2, 16, 12, 12, device=DEV)
    with pytest.raises(RuntimeError, match="does not match input channels"):
        _lib.conv_wgrad(x, gy, (16, 16, 3, 3), 1, 1)
    with pytest.raises(RuntimeError, match="grad_output shape"):
        _lib.conv_wgrad(x, torch.randn(2, 16, 11, 12, device=DEV), (16, 32, 3, 3), 1, 1)
    with pytest.raises(RuntimeError, match="grad_output shape"):
        _lib.conv_wgrad(x, torch.randn(2, 8, 12, 12, device=DEV), (16, 32, 3, 3), 1, 1)


WGRAD_SHAPES = [  # N, C, H, W, K, R, stride, pad, dilation
    (2, 3, 32, 32, 16, 3, 1, 1, 1),     # stem: C = 3
    (3, 16, 33, 30, 16, 3, 1, 1, 1),    # ragged rows, Q % 4 != 0 (scalar loads)
    (2, 48, 20, 20, 80, 3, 1, 1, 1),    # C, K past one 32-channel group, not multiples of 32
    (2, 16, 31, 31, 32, 3, 2, 1, 1),    # stride 2, odd sizes
    (2, 32, 28, 28, 64, 3, 2, 1, 1),    # stride 2, W % 4 == 0
    (2, 64, 14, 14, 16, 1, 1, 0, 1),    # 1x1 stride 1
    (2, 32, 15, 15, 64, 1, 2, 0, 1),    # 1x1 stride 2, ragged
    (2, 16, 12, 12, 16, 3, 1, 0, 1),    # 3x3 no padding
    (2, 16, 12, 12, 16, 3, 1, 2, 1),    # 3x3 padding 2
    (2, 16, 16, 16, 16, 3, 1, 2, 2),    # dilation 2 (LDS-band kernel)
    (1, 16, 8, 8, 16, 3, 1, 1, 1),      # fewer items than one block
]


@pytest.mark.parametrize("shape", WGRAD_SHAPES, ids=[str(s) for s in WGRAD_SHAPES])
def test_wgrad_kernels_vs_torch_fp64(shape):
    N, C, H, W, K, R, st, pad, dil = shape
    g = torch.Generator().manual_seed(sum(shape))
    x = torch.randn(N, C, H, W, generator=g)
    P = (H + 2 * pad - dil * (R - 1) - 1) // st + 1
    Q = (W + 2 * pad - dil * (R - 1) - 1) // st + 1
    gy = torch.randn(N, K, P, Q, generator=g)
    gw = _lib.conv_wgrad(x.to(DEV), gy.to(DEV), (K, C, R, R), st, pad, dil, 1)
    _, rw, _ = torch.ops.aten.convolution_backward(gy.double(), x.double(), torch.zeros(K, C, R, R, dtype=torch.float64),
                                                   None, [st, st], [pad, pad], [dil, dil], False, [0, 0], 1,
                                                   [False, True, False])
    assert nerr(gw, rw) <= CONV_TOL, nerr(gw, rw)


GROUPED = [  # N, C, H, W, K, R, stride, pad, dilation, groups, quantizer
    (2, 32, 16, 16, 32, 3, 1, 1, 1, 32, "po2+"),   # MobileNetV2 depthwise, stride 1
    (2, 96, 17, 17, 96, 3, 2, 1, 1, 96, "po2+"),   # depthwise stride 2, odd size
    (3, 144, 8, 8, 144, 3, 2, 1, 1, 144, "po2"),   # depthwise stride 2, even size
    (1, 24, 9, 13, 24, 5, 1, 2, 1, 24, "po2"),     # depthwise 5x5
    (2, 16, 12, 12, 32, 3, 1, 1, 1, 2, "po2"),     # grouped (input grad native, weight grad aten)
    (2, 16, 15, 15, 32, 3, 2, 1, 1, 1, "po2+"),    # dense stride 2, odd size
    (2, 8, 12, 12, 8, 3, 1, 2, 2, 1, "po2"),       # dilation 2
    (2, 16, 16, 16, 32, 1, 2, 0, 1, 1, None),      # 1x1 stride 2, plain weights
]


@pytest.mark.parametrize("shape", GROUPED, ids=[str(s) for s in GROUPED])
def test_grouped_strided_backward_vs_torch_fp64(shape):
    """Depthwise / grouped / strided / dilated layers: the input gradient through the forward
    kernels on zero-inserted dy, the depthwise weight gradient through its own kernel; against
    torch's fp64 CPU convolution_backward of Q(w).  Native unless marked (grouped non-depthwise
    weight gradients)."""
    from po2_quantization_amd.models import quantized_conv as qc

    N, C, H, W, K, R, st, pad, dil, groups, qn = shape
    g = torch.Generator().manual_seed(N * 7 + C + K + R)
    conv = QuantizedConv2d(C, K, R, stride=st, padding=pad, dilation=dil, groups=groups,
                           quantize_fn=quantizer_dict[qn] if qn else None, bits=4)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(conv.weight.shape, generator=g) * 0.3)
    conv = conv.to(DEV)
    x = torch.randn(N, C, H, W, generator=g).to(DEV).requires_grad_(True)
    before = qc.ATEN_BACKWARD_CALLS
    y = conv(x)
    gy = torch.randn(y.shape, generator=g).to(DEV)
    y.backward(gy)
    rx, rw, _ = ref_grads(x.detach(), conv.weight.detach(), None, gy, qn, 4, st, pad, groups, dil)
    assert nerr(x.grad, rx) <= CONV_TOL, nerr(x.grad, rx)
    assert nerr(conv.weight.grad, rw) <= CONV_TOL, nerr(conv.weight.grad, rw)
    dense_or_dw = groups == 1 or (groups == C == K)
    assert (qc.ATEN_BACKWARD_CALLS == before) == dense_or_dw


def test_reference_models_backward_all_native():
    """One QAT backward of ResNet20 and MobileNetV2 (CIFAR, po2+ 4-bit): no layer falls back to
    aten.convolution_backward (reference train.py:79-91)."""
    from po2_quantization_amd.models import quantized_conv as qc
    from po2_quantization_amd.models.model import get_model

    for mt in ("resnet20", "mobilenet"):
        m = get_model(mt, 10, quantizer_dict["po2+"], 4, (32, 32)).to(DEV).train()
        x = torch.randn(8, 3, 32, 32, device=DEV)
        before = qc.ATEN_BACKWARD_CALLS
        m(x).sum().backward()
        assert qc.ATEN_BACKWARD_CALLS == before, mt


@pytest.mark.parametrize("C,H,st", [(96, 32, 1), (144, 16, 2), (960, 4, 1)])
def test_depthwise_wgrad_full_size_vs_torch(C, H, st):
    """MobileNetV2 @32 depthwise layers at bs = 256: the depthwise weight gradient and the input
    gradient against torch's fp32 GPU convolution_backward of Q(w)."""
    torch.manual_seed(C)
    x = torch.randn(256, C, H, H, device=DEV)
    w = torch.randn(C, 1, 3, 3, device=DEV) * 0.3
    P = (H + 2 - 3) // st + 1
    gy = torch.randn(256, C, P, P, device=DEV)
    gw = _lib.conv_wgrad(x, gy, w.shape, st, 1, 1, C)
    qw = _lib.quantize(w, 4, "po2+")
    rx, rw, _ = torch.ops.aten.convolution_backward(gy, x, qw, None, [st, st], [1, 1], [1, 1], False, [0, 0], C,
                                                     [True, True, False])
    assert nerr(gw, rw) <= CONV_TOL, nerr(gw, rw)
    src = gy if st == 1 else _lib.dilate(gy, st, (H + 2 - 2, H + 2 - 2))
    gx = _lib.qconv2d(src, w.flip(2, 3).contiguous(), None, 1, 1, 1, C, 4, "po2+")
    assert nerr(gx, rx) <= CONV_TOL, nerr(gx, rx)


def test_dilate_zero_insertion():
    x = torch.randn(2, 3, 5, 4, device=DEV)
    for st, size in (((2, 2), (9, 7)), ((2, 3), (10, 11)), ((1, 1), (5, 4))):
        y = _lib.dilate(x, st, size)
        ref = torch.zeros(2, 3, *size, device=DEV)
        sub = ref[:, :, ::st[0], ::st[1]]
        h, w = min(sub.shape[2], 5), min(sub.shape[3], 4)
        ref[:, :, :h * st[0]:st[0], :w * st[1]:st[1]] = x[:, :, :h, :w]
        assert torch.equal(y, ref), st
