"""The drop-in on CPU tensors, with no stand-ins: the reference's QuantizedConv2d.forward runs on any
device (models/quantized_conv.py:32-38 -> F.conv2d), and BASELINE config 1 is a PTQ forward on CPU
(test.py:24-164).  Here QuantizedConv2d takes CPU input through its own torch path
(`_torch_forward`: the product's restated quantizers + torch's F.conv2d), never the oracle and never
libpo2q.  Checked against the golden outputs the reference produced (tests/golden/gen_golden.py).
"""
import numpy as np
import pytest
import torch

from po2_quantization_amd import _lib
from po2_quantization_amd.models.model import get_model
from po2_quantization_amd.models.quantized_conv import QuantizedConv2d
from po2_quantization_amd.utils.quantizers import quantize_model, quantizer_dict
from tests._util import CONV_TOL, GOLDEN, bits_equal, lin_kat_items, load_npz, normwise_err

import sys

sys.path.insert(0, GOLDEN)
from fill import seeded_fill_  # noqa: E402


@pytest.fixture(autouse=True)
def no_native(monkeypatch):
    """Any attempt to reach libpo2q / torch.ops.po2q from the CPU path fails the test."""
    def refuse(*a, **k):
        raise AssertionError("the CPU path reached the native library")
    monkeypatch.setattr(_lib, "load", refuse)
    monkeypatch.setattr(_lib, "ops", refuse)


def _resnet20_fp():
    m = get_model("resnet20", 10, None, 4, (32, 32))
    seeded_fill_(m, seed=7)
    return m.eval()


@pytest.mark.parametrize("qn", ["po2", "po2+", "lin", "lin+"])
def test_config1_ptq_resnet20_cpu(qn):
    """Config 1: ResNet20, quantize_model(model, quantizer, 4), then the eval forward on CPU, against
    the reference's PTQ error and logits (`ptq_err` / `ptq_logits` in models.npz)."""
    d = load_npz("models.npz")
    torch.set_num_threads(4)
    m = _resnet20_fp()
    err = quantize_model(m, quantizer_dict[qn], 4)
    ref_err = float(d["ptq_err/resnet20/%s/4" % qn])
    assert abs(err - ref_err) <= 1e-5 * ref_err, (err, ref_err)
    with torch.no_grad():
        y = m(torch.from_numpy(d["x/cifar8"])).numpy()
    e = normwise_err(y, d["ptq_logits/resnet20/%s/4" % qn])
    assert e <= CONV_TOL, e


MODELS = [("resnet20", None, 4), ("resnet56", "po2", 4), ("resnet20", "po2+", 3), ("mobilenet", "po2+", 4),
          ("mobilenet", "po2", 2), ("mobilevit", "po2+", 2), ("mobilevit", "po2", 4), ("mobilevit@64", "po2+", 2)]


@pytest.mark.parametrize("spec,q,bits", MODELS)
@pytest.mark.parametrize("train_mode", [False, True])
def test_qat_mode_logits_cpu(spec, q, bits, train_mode):
    """QAT-mode forwards (the weight quantized inside every conv's forward) of every model family on CPU
    against the reference's logits, in eval (the fused-call route falls back to the module sequence)
    and with autograd on (the plain module route)."""
    d = load_npz("models.npz")
    torch.set_num_threads(4)
    mt, _, sz = spec.partition("@")
    sz = int(sz or 32)
    m = get_model(mt, 10, quantizer_dict[q] if q else None, bits, (sz, sz))
    seeded_fill_(m, seed=7)
    m.eval()
    x = torch.from_numpy(d["x/cifar8"] if sz == 32 else d["x/img64"])
    with torch.set_grad_enabled(train_mode):
        y = m(x).detach().numpy()
    e = normwise_err(y, d["logits/%s/%s/%d" % (spec, q or "none", bits)])
    assert e <= CONV_TOL, e


def test_lin_quantizers_cpu_bit_exact():
    """restated_quantize_lin on CPU is the reference's arithmetic: bit for bit every lin / lin+ vector."""
    d, items = lin_kat_items()
    assert len(items) >= 200
    for key, name, qn, bits, iters, _ in items:
        x = torch.from_numpy(d["x/" + name])
        y = quantizer_dict[qn].apply(x, bits, iters).numpy()
        ok = bits_equal(y, d[key])
        assert ok.all(), (key, np.nonzero(~ok.ravel())[0][:8])


def test_conv_module_cpu_matches_torch_of_quantized_weight():
    """QuantizedConv2d on CPU == F.conv2d(x, Q(w)) with Q the restated quantizer, for strided, grouped,
    dilated and biased layers; the STE gradient reaches the weight."""
    g = torch.Generator().manual_seed(3)
    for kw in (dict(stride=1), dict(stride=2), dict(groups=4), dict(dilation=2, padding=2), dict(bias=True)):
        conv = QuantizedConv2d(8, 8, 3, quantize_fn=quantizer_dict["po2+"], bits=3, **kw)
        x = torch.randn(2, 8, 9, 11, generator=g, requires_grad=True)
        y = conv(x)
        qw = _lib.restated_quantize(conv.weight.detach(), 3, "po2+")
        ref = torch.nn.functional.conv2d(x.detach(), qw, conv.bias, conv.stride, conv.padding, conv.dilation,
                                         conv.groups)
        assert torch.equal(y.detach(), ref)
        y.sum().backward()
        assert conv.weight.grad is not None and x.grad is not None


def test_fused_calls_cpu_equal_module_sequence():
    """QuantizedConv2d.fused on CPU (the blocks' eval route) == conv -> bn -> + residual -> act."""
    g = torch.Generator().manual_seed(5)
    conv = QuantizedConv2d(8, 8, 3, quantize_fn=quantizer_dict["po2"], bits=4)
    bn = torch.nn.BatchNorm2d(8)
    with torch.no_grad():
        bn.running_mean.uniform_(-1, 1, generator=g)
        bn.running_var.uniform_(0.5, 2, generator=g)
    bn.eval()
    x = torch.randn(2, 8, 7, 7, generator=g)
    r = torch.randn(2, 8, 7, 7, generator=g)
    with torch.no_grad():
        for act, fn in (("relu", torch.relu), ("relu6", torch.nn.functional.relu6),
                        ("silu", torch.nn.functional.silu), (None, lambda t: t)):
            assert torch.equal(conv.fused(x, bn=bn, act=act, residual=r), fn(bn(conv(x)) + r))


def test_cpu_path_imports_no_oracle():
    """The product package never imports the oracle (grep over its sources)."""
    import os

    root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "po2_quantization_amd")
    for dirpath, _, files in os.walk(root):
        for f in files:
            if f.endswith(".py"):
                text = open(os.path.join(dirpath, f)).read()
                assert "import oracle" not in text and "from oracle" not in text, f
