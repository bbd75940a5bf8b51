"""GPU: batched weight staging (torch.ops.po2q.qconv2d_pack_batch + qconv2d_packed).
The batched launches quantize + pack exactly what each layer's own call would (same plan, same
kernel), so every result is bit for bit the per-layer call's; the model forwards with BATCHED_PACKS
on equal the forwards with it off."""
import pytest
import torch

from po2_quantization_amd import _lib
from po2_quantization_amd.models import quantized_conv as qc
from po2_quantization_amd.models.model import get_model
from po2_quantization_amd.utils.quantizers import quantizer_dict

pytestmark = pytest.mark.gpu
DEV = "cuda:0"

# (x shape, K, R, stride, pad, groups): stage-3 3x3 row kernel, stride-2 3x3, 1x1 stride-2 shortcut,
# MobileNetV2 pointwise expand / project, depthwise s1 / s2, a 5x5 and a ragged 3x3
LAYERS = [((4, 64, 14, 14), 64, 3, 1, 1, 1), ((4, 32, 28, 28), 64, 3, 2, 1, 1), ((4, 32, 28, 28), 64, 1, 2, 0, 1),
          ((8, 24, 8, 8), 144, 1, 1, 0, 1), ((8, 144, 8, 8), 24, 1, 1, 0, 1), ((8, 144, 8, 8), 144, 3, 1, 1, 144),
          ((8, 96, 16, 16), 96, 3, 2, 1, 96), ((2, 8, 13, 11), 12, 5, 1, 2, 1), ((3, 16, 23, 37), 16, 3, 1, 1, 1)]


@pytest.mark.parametrize("mode,bits", [("po2", 4), ("po2+", 2), ("po2", 3)])
def test_pack_batch_equals_per_layer_calls(mode, bits):
    torch.manual_seed(bits)
    xs, ws, specs = [], [], []
    for xshape, K, R, st, pad, g in LAYERS:
        x = torch.randn(*xshape, device=DEV)
        w = torch.randn(K, xshape[1] // g, R, R, device=DEV) * 0.1
        xs.append(x)
        ws.append(w)
        specs.append((w, xshape, st, pad, 1, g))
    packs = _lib.pack_batch(specs, bits, mode)
    assert len(packs) == len(LAYERS)
    assert any(p.numel() > 0 for p in packs)
    for (xshape, K, R, st, pad, g), x, w, ws_ in zip(LAYERS, xs, ws, packs):
        ps = torch.rand(K, device=DEV) + 0.5
        pb = torch.randn(K, device=DEV)
        ref = _lib.qconv2d_fused(x, w, None, st, pad, 1, g, bits, mode, post_scale=ps, post_shift=pb, act="relu")
        y = _lib.qconv2d_packed(x, w, ws_, None, st, pad, 1, g, bits, mode, post_scale=ps, post_shift=pb, act="relu")
        assert torch.equal(y, ref), (xshape, K, R, st, g)


def test_packed_run_checks_workspace():
    x = torch.randn(2, 64, 14, 14, device=DEV)
    w = torch.randn(64, 64, 3, 3, device=DEV) * 0.1
    (ws,) = _lib.pack_batch([(w, x.shape, 1, 1, 1, 1)], 4, "po2")
    if ws.numel() == 0:
        pytest.skip("this shape's plan stages its own weight")
    with pytest.raises(_lib.Po2qError, match="workspace"):
        _lib.qconv2d_packed(x, w, ws[:16], None, 1, 1, 1, 1, 4, "po2")


@pytest.mark.parametrize("name,image,q,bits", [("resnet20", 64, "po2", 4), ("mobilenet", 32, "po2+", 4),
                                               ("mobilevit", 64, "po2+", 2)])
def test_model_forward_batched_packs_bit_exact(name, image, q, bits, monkeypatch):
    """The models' eval forwards: the first forward at a shape records the layers, later forwards pack
    them in batched launches up front; logits bit for bit those of the per-layer packs (the fused
    inverted-residual block, which sums in another order, is off here: tests/test_gpu_ir.py)."""
    monkeypatch.setattr(qc, "IR_FUSION", False)
    torch.manual_seed(0)
    m = get_model(name, 10, quantizer_dict[q], bits, (image, image)).to(DEV).eval()
    x = torch.randn(4, 3, image, image, device=DEV)
    monkeypatch.setattr(qc, "BATCHED_PACKS", False)
    with torch.no_grad():
        ref = m(x)
    monkeypatch.setattr(qc, "BATCHED_PACKS", True)
    calls = []
    orig = _lib.qconv2d_packed
    monkeypatch.setattr(_lib, "qconv2d_packed", lambda *a, **k: calls.append(1) or orig(*a, **k))
    with torch.no_grad():
        y1 = m(x)  # records
        y2 = m(x)  # packs up front
        y3 = m(x)
    assert torch.equal(y1, ref) and torch.equal(y2, ref) and torch.equal(y3, ref)
    assert len(calls) > 0, "no layer ran from a batched pack"
    # a replaced weight is picked up (the pack is redone every forward, the module re-read)
    conv = next(c for c in m.modules() if isinstance(c, qc.QuantizedConv2d))
    conv.weight = torch.nn.Parameter(conv.weight.detach() * 2)
    monkeypatch.setattr(qc, "BATCHED_PACKS", False)
    with torch.no_grad():
        ref2 = m(x)
    monkeypatch.setattr(qc, "BATCHED_PACKS", True)
    with torch.no_grad():
        assert torch.equal(m(x), ref2)


@pytest.mark.parametrize("change", ["bits", "precision", "mode"])
def test_model_forward_repacks_when_layer_conf_changes(change, monkeypatch):
    """A layer's bits / quantizer / precision changed between two forwards at one input shape: the
    next forward must not run from a pack made for the old setting: it equals the
    per-layer forward of the new setting bit for bit."""
    torch.manual_seed(3)
    m = get_model("mobilenet", 10, quantizer_dict["po2"], 4, (32, 32)).to(DEV).eval()
    x = torch.randn(4, 3, 32, 32, device=DEV)
    with torch.no_grad():
        m(x)  # records
        m(x)  # packs up front
    convs = [c for c in m.modules() if isinstance(c, qc.QuantizedConv2d)]
    for c in convs[len(convs) // 2:]:
        if change == "bits":
            c.bits = 2
        elif change == "mode":
            c.quantize_fn = quantizer_dict["po2+"]
    if change == "precision":
        monkeypatch.setattr(qc.QuantizedConv2d, "precision", "fp32")
    monkeypatch.setattr(qc, "BATCHED_PACKS", False)
    with torch.no_grad():
        ref = m(x)
    monkeypatch.setattr(qc, "BATCHED_PACKS", True)
    with torch.no_grad():
        y1 = m(x)
        y2 = m(x)
    # IR_FUSION sums the fused blocks in another order than the layer calls: bit-exact only without it
    tol = 0.0 if not qc.IR_FUSION else 1e-5
    for y in (y1, y2):
        err = ((y - ref).abs().max() / ref.abs().max()).item()
        assert err <= tol, (change, err)


def test_session_ignores_modules_of_other_models():
    """A forward of another model inside an active session (a module of a different model, e.g. a
    DataParallel replica or a nested call) neither joins nor reads the first model's packs."""
    torch.manual_seed(4)
    a = get_model("resnet20", 10, quantizer_dict["po2"], 4, (64, 64)).to(DEV).eval()
    b = get_model("resnet20", 10, quantizer_dict["po2"], 4, (64, 64)).to(DEV).eval()
    x = torch.randn(2, 3, 64, 64, device=DEV)
    with torch.no_grad():
        ref_b = b(x)
        with qc.batched_packs(a, x):
            sess = qc._tls.packs
            yb = b(x)  # b's layers are not a's: no recording, no pack lookups
        assert sess.recording == []
        assert torch.equal(yb, ref_b)


@pytest.mark.parametrize("name,image", [("mobilenet", 32), ("mobilevit", 64)])
def test_batched_packs_see_weight_updates_and_graph_capture(name, image):
    """The batched packs re-quantize every forward: an in-place weight update queued just before a
    forward is seen (logits equal those of the per-layer packs); the forward captures into a HIP graph
    whose replays match."""
    torch.manual_seed(5)
    m = get_model(name, 10, quantizer_dict["po2+"], 4, (image, image)).to(DEV).eval()
    x = torch.randn(8, 3, image, image, device=DEV)
    with torch.no_grad():
        m(x)
        before = m(x)
        convs = [c for c in m.modules() if isinstance(c, qc.QuantizedConv2d)]
        for c in convs:
            c.weight.mul_(0.5)
        y = m(x)
        qc.BATCHED_PACKS = False
        try:
            ref2 = m(x)  # every layer packs its own (updated) weight
        finally:
            qc.BATCHED_PACKS = True
        # the per-layer path may pick other (fused-staging) plans: equal within the conv bar, and far
        # from the logits of the weights before the update
        err = lambda a, b: ((a - b).abs().max() / b.abs().max()).item()  # noqa: E731
        assert err(y, ref2) <= 1e-5 and err(before, ref2) > 1e-2
        ref2 = y
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            m(x)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = m(x)
        for _ in range(2):
            g.replay()
            torch.cuda.synchronize()
            assert torch.equal(out, ref2)


def test_replica_records_its_own_packs(monkeypatch):
    """A DataParallel-style replica (torch.nn.parallel.replicate: new module objects made from a shallow
    copy of the original's attributes) keeps its own layer record: its first forward records
    its own layers, and from its second forward on every layer that reads a pack in the original model's
    forwards reads one from the replica's own batched launch (the lookups key on the replica's modules)."""
    monkeypatch.setattr(qc, "IR_FUSION", False)
    torch.manual_seed(6)
    m = get_model("resnet20", 10, quantizer_dict["po2"], 4, (64, 64)).to(DEV).eval()
    x = torch.randn(2, 3, 64, 64, device=DEV)
    calls = []
    real_packed = _lib.qconv2d_packed

    def spy_packed(*a, **k):
        calls.append(1)
        return real_packed(*a, **k)

    monkeypatch.setattr(_lib, "qconv2d_packed", spy_packed)
    with torch.no_grad():
        m(x)
        del calls[:]
        ref = m(x)
        n_orig = len(calls)
        rep = torch.nn.parallel.replicate(m, [0], detach=True)[0]
        assert rep is not m
        del calls[:]
        y1 = rep(x)  # records the replica's layers
        n_first = len(calls)
        del calls[:]
        y2 = rep(x)  # reads its own batched packs
        n_second = len(calls)
    assert n_orig > 0 and n_first == 0 and n_second == n_orig, (n_orig, n_first, n_second)
    assert torch.equal(y1, ref) and torch.equal(y2, ref)
