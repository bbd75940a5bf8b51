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


def test_chain_and_pack_ops_registered_with_meta_shapes():
    """qconv2d_chain (a stage's stride-1 run in one launch), qconv2d_pack_batch (the batched weight
    staging of a forward) and qconv2d_packed (a conv from that workspace) are torch.ops with Meta
    kernels: the output shapes F.conv2d gives, one workspace per layer."""
    O = _lib.ops()
    x = torch.empty(4, 16, 32, 32, device="meta")
    ws = [torch.empty(16, 16, 3, 3, device="meta") for _ in range(3)]
    assert O.qconv2d_chain(x, ws, 4, 1, 1, [], [], [], [1, 1, 1], [-1, 0, -1]).shape == x.shape
    assert "Tensor[] weights" in str(O.qconv2d_chain.default._schema)
    # two layers: a stage-3 3x3 (a row kernel reading a packed weight) and a depthwise 3x3
    w3 = torch.empty(64, 64, 3, 3, device="meta")
    wd = torch.empty(96, 1, 3, 3, device="meta")
    geom = [256, 64, 56, 56, 1, 1, 1, 1, 1, 1, 1] + [8, 96, 16, 16, 1, 1, 1, 1, 1, 1, 96]
    out = O.qconv2d_pack_batch([w3, wd], geom, 4, 1, 1, 0, [-1, -1])
    assert len(out) == 2 and all(t.dtype == torch.uint8 and t.dim() == 1 for t in out)
    xs = torch.empty(256, 64, 56, 56, device="meta")
    y = O.qconv2d_packed(xs, w3, out[0], None, [1, 1], [1, 1], [1, 1], 1, 4, 1, 1, 0, -1, None, None, None, 1)
    assert y.shape == torch.nn.functional.conv2d(xs, w3, None, 1, 1).shape
    with pytest.raises(RuntimeError, match="bad lists|11 geometry"):
        O.qconv2d_pack_batch([w3], geom, 4, 1)


def test_chain_list_lengths_checked():
    """a per-layer list shorter or longer than the weights is an error (it was silently
    zero-filled: act none, no epilogue, res_from 0 = 'add x')."""
    x = torch.empty(2, 16, 8, 8)
    w = [torch.empty(16, 16, 3, 3)] * 3
    for kw in ({"acts": ["relu"] * 2}, {"res_from": [-1, 0]}, {"biases": [None] * 4}, {"post_scales": []}):
        with pytest.raises(_lib.Po2qError, match="one entry per weight"):
            _lib.qconv2d_chain(x, w, **kw)


@pytest.mark.parametrize("Cin,Ch,Cout,H,stride,expand", [(16, 96, 24, 16, 2, True), (32, 32, 16, 16, 1, False),
                                                          (160, 960, 320, 1, 1, True), (12, 80, 20, 9, 2, True)])
def test_ir_op_meta_shape(Cin, Ch, Cout, H, stride, expand):
    """qconv2d_ir (a whole inverted-residual block in one launch): the project conv's output shape
    of the depthwise conv's output, as the three F.conv2d calls give it."""
    O = _lib.ops()
    x = torch.empty(3, Cin, H, H, device="meta")
    we = torch.empty(Ch, Cin, 1, 1, device="meta") if expand else None
    wd = torch.empty(Ch, 1, 3, 3, device="meta")
    wp = torch.empty(Cout, Ch, 1, 1, device="meta")
    ws = torch.empty(0, dtype=torch.uint8, device="meta")
    y = O.qconv2d_ir(x, we, wd, wp, ws if expand else None, ws, ws, stride, 4, 1)
    F = torch.nn.functional
    h = F.conv2d(x, we) if expand else x
    want = F.conv2d(F.conv2d(h, wd, None, stride, 1, 1, Ch), wp).shape
    assert y.shape == want
    with pytest.raises(RuntimeError, match="project weight"):
        O.qconv2d_ir(x, we, wd, torch.empty(Cout, Ch + 1, 1, 1, device="meta"), ws if expand else None, ws, ws,
                     stride, 4, 1)


def test_ir_block_detection():
    """The models' inverted-residual conv blocks are recognised for the fused launch; a quantizer-free
    block (mode none: nothing to pack) and a 3x3-conv block are not."""
    from po2_quantization_amd.models import quantized_conv as qc
    from po2_quantization_amd.models.mobilenet import InvertedResidual
    from po2_quantization_amd.utils.quantizers import quantizer_dict

    q = quantizer_dict["po2"]
    blk = InvertedResidual(24, 24, 1, 6, quantize_fn=q)
    e, d, p = qc._ir_spec(blk.conv)
    assert e[2] == "relu6" and d[2] == "relu6" and p[2] is None and d[0].groups == 144
    blk1 = InvertedResidual(32, 16, 1, 1, quantize_fn=q)
    e, d, p = qc._ir_spec(blk1.conv)
    assert e is None and d[0].groups == 32
    assert qc._ir_spec(InvertedResidual(24, 24, 1, 6, quantize_fn=None).conv) is None
    from po2_quantization_amd.models.mobilenet import quantized_conv_3x3_bn
    assert qc._ir_spec(quantized_conv_3x3_bn(16, 16, 1, quantize_fn=q)) is None
