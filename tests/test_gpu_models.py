"""GPU parity at model level: the drop-in modules inside the reference's model
graphs reproduce the reference's logits (golden vectors from running the
reference models on CPU, tests/golden/gen_golden.py) on identical weights."""
import os
import sys

import numpy as np
import pytest
import torch

from po2_quantization_amd.models.model import get_model
from po2_quantization_amd.utils.quantizers import quantize_model, quantizer_dict
from tests._util import CONV_TOL, GOLDEN, load_npz, normwise_err

sys.path.insert(0, GOLDEN)
from fill import seeded_fill_  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
# logits go through ~57 conv layers + BN; per-layer normwise error ~1e-7 → allow 1e-5 on logits
LOGIT_TOL = CONV_TOL


def build(spec, q, bits):
    mt, _, sz = spec.partition("@")
    m = get_model(mt, 10, quantizer_dict[q] if q else None, bits, (int(sz or 32),) * 2)
    seeded_fill_(m, seed=7)
    return m.to(DEV).eval()


# config 2 (resnet56 po2-4), config 3 (mobilenet po2+-4: depthwise + pointwise convs),
# config 5 (mobilevit po2+-2, weights only; @64 = the 2x2-patch path used at ImageNet sizes)
@pytest.mark.parametrize("spec,q,bits", [("resnet20", None, 4), ("resnet56", "po2", 4), ("resnet20", "po2+", 3),
                                         ("mobilenet", "po2+", 4), ("mobilenet", "po2", 2),
                                         ("mobilevit", "po2+", 2), ("mobilevit", "po2", 4),
                                         ("mobilevit@64", "po2+", 2)])
def test_qat_mode_logits(spec, q, bits, monkeypatch):
    """Three eval forwards at one shape: the first records which layers read a packed weight
    (models/quantized_conv.py batched_packs), the later ones run the path the bench and users run
    from then on -- the batched weight packs and, for MobileNetV2, the fused inverted-residual block
    kernel at its 4x4 blocks (asserted to run).  Every forward's logits against the reference's."""
    from po2_quantization_amd import _lib

    calls = {"ir": 0, "packed": 0}
    ir, packed = _lib.qconv2d_ir, _lib.qconv2d_packed
    monkeypatch.setattr(_lib, "qconv2d_ir", lambda *a, **k: calls.__setitem__("ir", calls["ir"] + 1) or ir(*a, **k))
    monkeypatch.setattr(_lib, "qconv2d_packed",
                        lambda *a, **k: calls.__setitem__("packed", calls["packed"] + 1) or packed(*a, **k))
    d = load_npz("models.npz")
    m = build(spec, q, bits)
    x = torch.from_numpy(d["x/img64"] if spec.endswith("@64") else d["x/cifar8"]).to(DEV)
    ref = d["logits/%s/%s/%d" % (spec, q or "none", bits)]
    with torch.no_grad():
        y1 = m(x).cpu().numpy()
        assert calls == {"ir": 0, "packed": 0}  # the recording forward: per-layer calls
        y2 = m(x).cpu().numpy()
        y3 = m(x).cpu().numpy()
    for y in (y1, y2, y3):
        assert normwise_err(y, ref) <= LOGIT_TOL, normwise_err(y, ref)
    if q is not None:
        assert calls["packed"] > 0, calls  # the second forward ran from the batched packs
    if spec == "mobilenet":
        assert calls["ir"] >= 2, calls  # the 4x4 blocks as one qconv2d_ir launch each, in both later forwards


@pytest.mark.parametrize("spec,q,bits,n", [("resnet56", "po2", 4, 9), ("resnet20", "po2+", 3, 3)])
def test_cifar_resnet_logits_through_chain_kernel(spec, q, bits, n, monkeypatch):
    """At CIFAR size the eval forward runs each stage's identity-shortcut blocks as ONE chain launch
    (po2q_qconv2d_chain_f32: stage 1 all n blocks, stages 2-3 the n - 1 after the transition); the
    logits still match the reference's (reference resnet.py:55-71, 190-201)."""
    from po2_quantization_amd import _lib

    calls = []
    orig = _lib.qconv2d_chain

    def counted(x, ws, *a, **k):
        calls.append(len(ws))
        return orig(x, ws, *a, **k)

    monkeypatch.setattr(_lib, "qconv2d_chain", counted)
    d = load_npz("models.npz")
    m = build(spec, q, bits)
    with torch.no_grad():
        y = m(torch.from_numpy(d["x/cifar8"]).to(DEV)).cpu().numpy()
    assert calls == [2 * n, 2 * (n - 1), 2 * (n - 1)], calls
    ref = d["logits/%s/%s/%d" % (spec, q, bits)]
    assert normwise_err(y, ref) <= LOGIT_TOL, normwise_err(y, ref)


@pytest.mark.parametrize("qn", ["po2", "po2+", "lin", "lin+"])
def test_ptq_config1_resnet20(qn):
    """Config 1 (test.py PTQ path): quantize_model(model, quantizer, 4) then eval."""
    d = load_npz("models.npz")
    m = build("resnet20", None, 4)
    err = quantize_model(m, quantizer_dict[qn], 4)
    ref_err = float(d["ptq_err/resnet20/%s/4" % qn])
    assert abs(err - ref_err) <= 1e-5 * ref_err, (err, ref_err)
    with torch.no_grad():
        y = m(torch.from_numpy(d["x/cifar8"]).to(DEV)).cpu().numpy()
    assert normwise_err(y, d["ptq_logits/resnet20/%s/4" % qn]) <= LOGIT_TOL


def test_state_dict_keys_match_reference():
    import json

    keys = json.load(open(os.path.join(GOLDEN, "models.json")))
    for mt in ("resnet20", "resnet56", "mobilenet", "mobilevit"):
        m = get_model(mt, 10, None, 4, (32, 32))
        assert [[k, list(v.shape)] for k, v in m.state_dict().items()] == keys[mt]


@pytest.mark.parametrize("spec,q,bits", [("resnet56", "po2", 4), ("resnet20", "po2+", 3), ("mobilenet", "po2+", 4),
                                         ("mobilenet", "po2", 2), ("mobilevit", "po2+", 2), ("mobilevit", "po2", 4)])
def test_model_quantization_error_through_hip_quantizer(spec, q, bits):
    """get_quantization_error (models/quantized_conv.py:40-45, model-level sums with the
    reference's counting quirks) through the HIP quantizer == the reference's values."""
    d = load_npz("models.npz")
    m = build(spec, q, bits)
    e, n = m.get_quantization_error()
    ref_e, ref_n = d["qerr/%s/%s/%d" % (spec, q, bits)]
    assert int(n) == int(ref_n)
    assert abs(float(torch.as_tensor(e).detach().cpu()) - ref_e) <= 1e-5 * ref_e


def test_layer_quantization_error_vs_oracle():
    """QuantizedConv2d.get_quantization_error on GPU: (sum (Q(w) - w)^2, numel), Q bit-exact."""
    from oracle import oracle as O
    from po2_quantization_amd.models.quantized_conv import QuantizedConv2d

    g = torch.Generator().manual_seed(5)
    for qn in ("po2", "po2+"):
        conv = QuantizedConv2d(32, 64, 3, quantize_fn=quantizer_dict[qn], bits=4)
        with torch.no_grad():
            conv.weight.copy_(torch.randn(conv.weight.shape, generator=g) * 0.05)
        conv = conv.to(DEV)
        e, n = conv.get_quantization_error()
        w = conv.weight.detach().cpu().numpy()
        ref = O.sq_error(w, O.quantize(w, 4, qn))
        assert int(n) == w.size
        assert abs(float(torch.as_tensor(e).detach().cpu()) - ref) <= 1e-5 * ref  # fp32 sum (torch) vs fp64


@pytest.mark.parametrize("tag", ["resnet56@128/po2/4", "resnet20@224/po2+/4"])
@pytest.mark.parametrize("pair_c32", [False, True])
def test_wide_resnet_logits_through_fused_block_kernels(tag, pair_c32, monkeypatch):
    """Reference logits (tests/golden/models_wide.npz, generated by running the reference's
    ResNet, models/resnet.py:55-71,150-163,190-201) through the drop-in's eval forward at a width
    where BasicBlock.forward takes the fused-block kernels: the stage-1 conv pair, the stage-2 pairs
    (advised by default; PO2Q_PAIR_C32=0 turns them off) and the stride-2 + shortcut kernel.  Asserts
    they ran."""
    from po2_quantization_amd import _lib

    monkeypatch.setenv("PO2Q_PAIR_C32", "1" if pair_c32 else "0")  # stage-2 pairs advised by default
    d = load_npz("models_wide.npz")
    spec, q, bits = tag.split("/")
    mt, sz = spec.split("@")
    m = get_model(mt, 10, quantizer_dict[q], int(bits), (int(sz),) * 2)
    seeded_fill_(m, seed=7)
    m = m.to(DEV).eval()
    calls = {"pair16": 0, "pair32": 0, "s2ds": 0}
    pair, s2ds = _lib.qconv2d_pair, _lib.qconv2d_s2ds

    def count_pair(x, *a, **k):
        calls["pair%d" % x.shape[1]] += 1
        return pair(x, *a, **k)

    def count_s2ds(*a, **k):
        calls["s2ds"] += 1
        return s2ds(*a, **k)

    monkeypatch.setattr(_lib, "qconv2d_pair", count_pair)
    monkeypatch.setattr(_lib, "qconv2d_s2ds", count_s2ds)
    nb = len(m.layer1)
    with torch.no_grad():
        y = m(torch.from_numpy(d["x/" + tag]).to(DEV)).cpu().numpy()
    assert calls["pair16"] == nb and calls["s2ds"] >= 1, calls
    assert calls["pair32"] == (nb - 1 if pair_c32 else 0), calls
    assert normwise_err(y, d["logits/" + tag]) <= LOGIT_TOL, normwise_err(y, d["logits/" + tag])


def test_mobilevit_256_logits_config5(monkeypatch):
    """BASELINE config 5 at its own size: MobileViT-XS @256x256, 1000 classes, po2+ 2-bit QAT-mode
    weights (the reference quantizes no activations), eval forward with every conv + BN + act native,
    against the reference's logits (tests/golden/models_vit256.npz; reference models/mobile_vit.py:
    131-311).  The input comes from its seed (torch CPU generator), checked by its sum."""
    d = load_npz("models_vit256.npz")
    tag = "mobilevit@256/po2+/2"
    x = torch.randn(2, 3, 256, 256, generator=torch.Generator().manual_seed(5))
    assert abs(float(x.double().sum()) - float(d["x_sum/" + tag])) <= 1e-6 * abs(float(d["x_sum/" + tag])) + 1e-3
    m = get_model("mobilevit", 1000, quantizer_dict["po2+"], 2, (256, 256))
    seeded_fill_(m, seed=7)
    m = m.to(DEV).eval()
    from po2_quantization_amd import _lib

    n = [0]
    packed = _lib.qconv2d_packed
    monkeypatch.setattr(_lib, "qconv2d_packed", lambda *a, **k: n.__setitem__(0, n[0] + 1) or packed(*a, **k))
    with torch.no_grad():
        y1 = m(x.to(DEV)).cpu().numpy()  # records
        y2 = m(x.to(DEV)).cpu().numpy()  # batched packs (the path config 5's bench replays)
    assert n[0] > 0
    for y in (y1, y2):
        assert normwise_err(y, d["logits/" + tag]) <= LOGIT_TOL, normwise_err(y, d["logits/" + tag])
