"""conv_rowsk's pipelined split (PIPE: the split of halo row j + 1 beside row j's MFMAs, one barrier
at the end of each step; po2q_conv_rowsk.hip) against the one-row-at-a-time kernel: bit for bit on
every C = K = 64 row-kernel plan, full and ragged shapes, with and without the fused epilogue, and
against torch's fp32 conv of the quantized weight (the reference's QuantizedConv2d.forward,
models/quantized_conv.py:32-38) within the conv tolerance."""
import re

import pytest
import torch
import torch.nn.functional as F

from po2_quantization_amd import _lib
from tests._util import CONV_TOL

pytestmark = pytest.mark.gpu

SHAPES = [(2, 56, 56), (3, 13, 12), (2, 20, 28), (1, 9, 44), (4, 30, 8), (1, 57, 12)]


def rowsk_plans(n, h, w):
    ds = _lib.plans(n, 64, h, w, 64, 3, 3, 1, 1)
    return [i for i, d in enumerate(ds) if "bf16x3_rows" in d and "CC=32" in d and re.search(r"\bfp=0\b", d)
            and re.search(r"\bvr=[12]\b", d)]


@pytest.mark.parametrize("shape", SHAPES)
def test_rowsk_pipe_bitwise(shape, monkeypatch):
    n, h, w_ = shape
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(h * 131 + w_)
    x = torch.relu(torch.randn(n, 64, h, w_, device=dev, generator=g))
    w = torch.randn(64, 64, 3, 3, device=dev, generator=g) * 0.05
    ps = torch.rand(64, device=dev, generator=g) + 0.5
    pb = torch.randn(64, device=dev, generator=g) * 0.1
    idx = rowsk_plans(n, h, w_)
    assert idx, "no row-kernel plan for this shape"
    ref = F.conv2d(x, _lib.quantize(w, 4, "po2"), None, 1, 1)
    for i in idx:
        outs = []
        ws = _lib.pack_batch([(w, tuple(x.shape), 1, 1, 1, 1)], plans=[i])[0]
        for pipe in ("0", "1"):
            monkeypatch.setenv("PO2Q_ROWSK_PIPE", pipe)
            outs.append((_lib.qconv2d(x, w, None, 1, 1, 1, 1, 4, "po2", plan=i),
                         _lib.qconv2d_packed(x, w, ws, None, 1, 1, 1, 1, 4, "po2", post_scale=ps, post_shift=pb,
                                             act="relu", plan=i)))
        torch.cuda.synchronize()
        assert torch.equal(outs[0][0], outs[1][0]), (shape, i)
        assert torch.equal(outs[0][1], outs[1][1]), (shape, i)
        err = (outs[1][0] - ref).abs().max() / ref.abs().max()
        assert err <= CONV_TOL, (shape, i, float(err))
