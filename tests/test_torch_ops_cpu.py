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
