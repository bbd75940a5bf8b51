"""CPU: the PyTorch-ROCm operator library (torch.ops.po2q, csrc/po2q_torch.cpp) loads,
registers its schemas, gives F.conv2d's output shapes through its Meta kernels, and
refuses CPU tensors (no CPU path).  No GPU needed."""
import pytest
import torch

from po2_quantization_amd import _lib


def test_ops_registered():
    O = _lib.ops()
    for name in ("quantize", "quantize_lin", "qconv2d", "qconv2d_fused"):
        assert hasattr(O, name), name
    s = str(O.qconv2d.default._schema)
    assert "Tensor? bias" in s and "int[2] stride" in s


@pytest.mark.parametrize("shape", [(2, 16, 32, 32, 16, 3, 1, 1), (2, 16, 33, 31, 32, 3, 2, 1),
                                   (3, 32, 16, 16, 64, 1, 2, 0), (1, 8, 70, 70, 24, 3, 1, 1)])
def test_meta_shapes_match_conv2d(shape):
    N, C, H, K, W, R, st, pad = shape[0], shape[1], shape[2], shape[4], shape[3], shape[5], shape[6], shape[7]
    x = torch.empty(N, C, H, W, device="meta")
    w = torch.empty(K, C, R, R, device="meta")
    want = torch.nn.functional.conv2d(x, w, None, st, pad).shape
    O = _lib.ops()
    assert O.qconv2d(x, w, None, [st, st], [pad, pad], [1, 1], 1, 4, 1).shape == want
    assert O.qconv2d_fused(x, w, None, [st, st], [pad, pad], [1, 1], 1, 4, 2, act=1).shape == want
    assert O.quantize(w, 4, 1).shape == w.shape


def test_cpu_tensors_have_no_kernel():
    O = _lib.ops()
    with pytest.raises(RuntimeError):
        O.qconv2d(torch.randn(1, 4, 8, 8), torch.randn(4, 4, 3, 3), None, [1, 1], [1, 1], [1, 1], 1, 4, 1)


@pytest.mark.parametrize("C,H,W", [(16, 224, 224), (32, 112, 112), (16, 17, 8)])
def test_s2ds_meta_shapes_match_both_convs(C, H, W):
    """qconv2d_s2ds: the 3x3 s2 p1 conv and the 1x1 s2 conv of the same x have one output shape."""
    x = torch.empty(2, C, H, W, device="meta")
    w = torch.empty(2 * C, C, 3, 3, device="meta")
    wds = torch.empty(2 * C, C, 1, 1, device="meta")
    y, yds = _lib.ops().qconv2d_s2ds(x, w, wds, 4, 1)
    assert y.shape == torch.nn.functional.conv2d(x, w, None, 2, 1).shape
    assert yds.shape == torch.nn.functional.conv2d(x, wds, None, 2, 0).shape
