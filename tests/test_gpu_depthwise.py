"""GPU parity of the depthwise 3x3 kernels (MobileNetV2 inverted-residual depthwise layers,
reference models/mobilenet.py:64-76 -> QuantizedConv2d(groups=hidden_dim), quantized_conv.py:
32-38): the LDS-halo kernel (plan 0) and the one-output-per-lane kernel (plan 1) against the
fp64 oracle, plain and with the fused eval-BN + ReLU6 (+ residual) epilogue against torch fp32.
Bar: normwise 1e-5 (CONV_TOL)."""
import pytest
import torch

from oracle import oracle as O
from po2_quantization_amd import _lib
from tests._util import CONV_TOL, normwise_err

pytestmark = pytest.mark.gpu
DEV = "cuda:0"

DW_SHAPES = [  # N, C, H, W, stride
    (2, 96, 32, 32, 1),    # MobileNetV2 @32: expansion of 16
    (2, 144, 32, 32, 2),   # stride-2 depthwise
    (3, 192, 16, 16, 1),
    (2, 384, 8, 8, 1),
    (2, 960, 4, 4, 1),
    (2, 576, 8, 8, 2),     # -> 4x4
    (1, 32, 112, 112, 1),  # @224 stage: several row bands
    (1, 24, 57, 57, 2),    # odd sizes, W % 4 != 0 (scalar staging / stores)
    (2, 40, 30, 30, 1),    # W % 4 != 0, Q % 4 != 0
    (1, 8, 1, 1, 1),       # one pixel
    (1, 8, 2, 3, 2),
]


@pytest.mark.parametrize("shape", DW_SHAPES, ids=[str(s) for s in DW_SHAPES])
def test_depthwise_every_plan_vs_oracle(shape):
    N, C, H, W, st = shape
    g = torch.Generator().manual_seed(hash(shape) & 0xFFFF)
    x = torch.randn(N, C, H, W, generator=g)
    w = torch.randn(C, 1, 3, 3, generator=g) * 0.3
    b = torch.randn(C, generator=g) * 0.1
    ref, _ = O.qconv2d(x.numpy(), w.numpy(), b.numpy(), st, 1, 1, C, 4, "po2+")
    plans = _lib.plans(N, C, H, W, C, 3, 3, st, 1, 1, C, 4, "po2+")
    assert "kind=depthwise" in plans[0] and "vr=1" in plans[0], plans[0]
    assert len(plans) == 2 and "vr=0" in plans[1]
    xd, wd, bd = x.to(DEV), w.to(DEV), b.to(DEV)
    for i, desc in enumerate(plans):
        y = _lib.qconv2d(xd, wd, bd, st, 1, 1, C, 4, "po2+", plan=i).cpu().numpy()
        assert normwise_err(y, ref) <= CONV_TOL, (desc, normwise_err(y, ref))


def test_depthwise_unaligned_views():
    """Input / output views that are not 16-byte aligned take the scalar paths."""
    torch.manual_seed(5)
    big = torch.randn(1 * 96 * 32 * 32 + 1, device=DEV)
    x = big[1:].view(1, 96, 32, 32)  # 4-byte offset
    w = torch.randn(96, 1, 3, 3, device=DEV) * 0.3
    y = _lib.qconv2d(x, w, None, 1, 1, 1, 96, 4, "po2")
    ref = torch.nn.functional.conv2d(x, _lib.quantize(w, 4, "po2"), None, 1, 1, 1, 96)
    assert ((y - ref).abs().max() / ref.abs().max()).item() <= CONV_TOL


@pytest.mark.parametrize("shape", [(2, 144, 16, 16, 1), (2, 144, 32, 32, 2), (1, 40, 30, 30, 1)])
@pytest.mark.parametrize("with_res", [False, True])
def test_depthwise_fused_bn_relu6(shape, with_res):
    N, C, H, W, st = shape
    g = torch.Generator().manual_seed(7 + st)
    x = torch.randn(N, C, H, W, generator=g).to(DEV)
    w = (torch.randn(C, 1, 3, 3, generator=g) * 0.3).to(DEV)
    ps = (torch.rand(C, generator=g) + 0.5).to(DEV)
    pb = (torch.randn(C, generator=g) * 0.1).to(DEV)
    qw = _lib.quantize(w, 4, "po2+")
    y0 = torch.nn.functional.conv2d(x, qw, None, st, 1, 1, C) * ps.view(1, -1, 1, 1) + pb.view(1, -1, 1, 1)
    res = torch.randn(y0.shape, generator=g).to(DEV) if with_res else None
    ref = torch.nn.functional.relu6(y0 + res if with_res else y0)
    y = _lib.qconv2d_fused(x, w, None, st, 1, 1, C, 4, "po2+", post_scale=ps, post_shift=pb, residual=res,
                           act="relu6")
    assert ((y - ref).abs().max() / ref.abs().max()).item() <= CONV_TOL
