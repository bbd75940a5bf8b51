"""GPU parity of the fused stride-2 transition (po2q_qconv2d_s2ds_f32): a stage's first-block
conv1 (QuantizedConv2d 3x3 stride 2, C -> 2C) and its projection shortcut downsample.0
(QuantizedConv2d 1x1 stride 2) on the same x in one launch (reference models/resnet.py:55-71,
each conv QuantizedConv2d.forward, models/quantized_conv.py:32-38), against torch fp32 convs of
the bit-exact Q(w) (a plain PyTorch fp32 reference) and against the single-conv path.
Bar: normwise 1e-5 (CONV_TOL)."""
import pytest
import torch
import torch.nn.functional as F

from po2_quantization_amd import _lib
from tests._util import CONV_TOL

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def nerr(y, ref):
    return ((y - ref).abs().max() / ref.abs().max()).item()


def make(N, C, H, W, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(N, C, H, W, generator=g).to(DEV)
    w = (torch.randn(2 * C, C, 3, 3, generator=g) * 0.1).to(DEV)
    wds = (torch.randn(2 * C, C, 1, 1, generator=g) * 0.2).to(DEV)
    return x, w, wds


SHAPES = [(2, 16, 40, 40), (1, 16, 9, 64), (1, 16, 17, 8), (2, 16, 30, 224), (3, 16, 2, 16),
          (2, 32, 40, 40), (1, 32, 17, 8), (2, 32, 30, 112), (1, 32, 1, 16)]


@pytest.mark.parametrize("shape", SHAPES, ids=[str(s) for s in SHAPES])
@pytest.mark.parametrize("mode", ["po2", "po2+"])
def test_s2ds_vs_torch(shape, mode):
    N, C, H, W = shape
    x, w, wds = make(N, C, H, W, hash(shape) & 0xFFFF)
    y, yds = _lib.qconv2d_s2ds(x, w, wds, 4, mode)
    ref = F.conv2d(x, _lib.quantize(w, 4, mode), None, 2, 1)
    refds = F.conv2d(x, _lib.quantize(wds, 4, mode), None, 2, 0)
    assert y.shape == ref.shape and yds.shape == refds.shape
    assert nerr(y, ref) <= CONV_TOL, nerr(y, ref)
    assert nerr(yds, refds) <= CONV_TOL, nerr(yds, refds)
    # the 3x3 output is the single-conv stride-2 kernel's, same bf16x3 arithmetic
    y1 = _lib.qconv2d(x, w, None, 2, 1, 1, 1, 4, mode)
    assert nerr(y, y1) <= 1e-6, nerr(y, y1)


@pytest.mark.parametrize("C", [16, 32])
def test_s2ds_epilogues_vs_torch(C):
    """Eval BatchNorm + ReLU on conv1, eval BatchNorm on the shortcut (BasicBlock's two branches)."""
    x, w, wds = make(2, C, 36, 64, 7 + C)
    g = torch.Generator().manual_seed(3)
    ps, psd = (torch.rand(2 * C, generator=g) + 0.5).to(DEV), (torch.rand(2 * C, generator=g) + 0.5).to(DEV)
    pb, pbd = (torch.randn(2 * C, generator=g) * 0.1).to(DEV), (torch.randn(2 * C, generator=g) * 0.1).to(DEV)
    y, yds = _lib.qconv2d_s2ds(x, w, wds, 4, "po2+", post_scale=ps, post_shift=pb, act="relu",
                               post_scale_ds=psd, post_shift_ds=pbd)
    v = lambda t: t.view(1, -1, 1, 1)  # noqa: E731
    ref = torch.relu(F.conv2d(x, _lib.quantize(w, 4, "po2+"), None, 2, 1) * v(ps) + v(pb))
    refds = F.conv2d(x, _lib.quantize(wds, 4, "po2+"), None, 2, 0) * v(psd) + v(pbd)
    assert nerr(y, ref) <= CONV_TOL, nerr(y, ref)
    assert nerr(yds, refds) <= CONV_TOL, nerr(yds, refds)


@pytest.mark.parametrize("C,H", [(16, 224), (32, 112)])
def test_s2ds_full_size(C, H):
    """BASELINE size (bs = 256): layer2.0 (16 -> 32 @224) and layer3.0 (32 -> 64 @112)."""
    torch.manual_seed(0)
    x = torch.relu(torch.randn(256, C, H, H, device=DEV))
    w = torch.randn(2 * C, C, 3, 3, device=DEV) * 0.1
    wds = torch.randn(2 * C, C, 1, 1, device=DEV) * 0.2
    y, yds = _lib.qconv2d_s2ds(x, w, wds, 4, "po2")
    ref = F.conv2d(x, _lib.quantize(w, 4, "po2"), None, 2, 1)
    assert nerr(y, ref) <= CONV_TOL, nerr(y, ref)
    del ref
    refds = F.conv2d(x, _lib.quantize(wds, 4, "po2"), None, 2, 0)
    assert nerr(yds, refds) <= CONV_TOL, nerr(yds, refds)
    # the bench's launch geometry against the fp64 oracle on sampled images (grid ends, other XCDs)
    from oracle import oracle as O

    idx = [0, 37, 130, 255]
    xs = x[idx].cpu().numpy()
    for out, wt, st, pad in ((y, w, 2, 1), (yds, wds, 2, 0)):
        o, _ = O.qconv2d(xs, wt.cpu().numpy(), None, st, pad, 1, 1, 4, "po2")
        err = abs(out[idx].cpu().numpy().astype("float64") - o).max() / abs(o).max()
        assert err <= CONV_TOL, err


def test_s2ds_rejects():
    assert not _lib.s2ds_supported((2, 64, 56, 56))
    # advisory: wide rows only (ResNet56 @224); CIFAR-size rows run two launches
    assert _lib.s2ds_supported((256, 16, 224, 224)) and _lib.s2ds_supported((256, 32, 112, 112))
    assert not _lib.s2ds_supported((256, 16, 32, 32)) and not _lib.s2ds_supported((256, 32, 16, 16))
    assert not _lib.s2ds_supported((2, 16, 40, 42))  # W % 4
    x = torch.randn(1, 64, 8, 8, device=DEV)
    with pytest.raises(_lib.Po2qError):
        _lib.qconv2d_s2ds(x, torch.randn(128, 64, 3, 3, device=DEV), torch.randn(128, 64, 1, 1, device=DEV))
    x = torch.randn(1, 16, 8, 8, device=DEV)
    with pytest.raises(_lib.Po2qError, match="shortcut weight"):
        _lib.qconv2d_s2ds(x, torch.randn(32, 16, 3, 3, device=DEV), torch.randn(32, 16, 3, 3, device=DEV))


@pytest.mark.parametrize("stage,C,H", [(2, 16, 112), (3, 32, 112)])
@pytest.mark.parametrize("q", ["po2", "po2+"])
def test_basicblock_eval_fused_equals_module_sequence(stage, C, H, q, monkeypatch):
    """ResNet56 layer{2,3}.0 in eval: BasicBlock.forward through qconv2d_s2ds (conv1 + BN + ReLU and
    the 1x1 shortcut + BN on one read of x) equals the plain module sequence."""
    from po2_quantization_amd.models import quantized_conv as qc
    from po2_quantization_amd.models.model import get_model
    from po2_quantization_amd.utils.quantizers import quantizer_dict

    m = get_model("resnet56", 10, quantizer_dict[q], 4, (32, 32))
    blk = getattr(m, "layer%d" % stage)[0]
    g = torch.Generator().manual_seed(stage)
    for bn in (blk.bn1, blk.bn2, blk.downsample[1]):
        bn.running_mean.copy_(torch.randn(bn.num_features, generator=g) * 0.1)
        bn.running_var.copy_(torch.rand(bn.num_features, generator=g) + 0.5)
        bn.weight.data.copy_(torch.rand(bn.num_features, generator=g) + 0.5)
        bn.bias.data.copy_(torch.randn(bn.num_features, generator=g) * 0.1)
    blk = blk.to(DEV).eval()
    x = torch.relu(torch.randn(4, C, H, H, generator=g)).to(DEV)
    assert blk._s2ds_ok(x)
    with torch.no_grad():
        y = blk(x)
        monkeypatch.setattr(qc, "INFERENCE_FUSION", False)
        ref = blk(x)
    assert nerr(y, ref) <= 1e-6, nerr(y, ref)


def test_packed_convs_equal_per_layer_calls():
    """_lib.PackedConvs (one batched weight-pack launch for every layer, then each conv from its
    packed workspace) gives qconv2d()'s results bit for bit, layer by layer (ResNet56 stage-2 /
    stage-3 shapes, a 1x1 stride-2 layer, and more layers than one 16-job launch holds)."""
    g = torch.Generator().manual_seed(11)
    shapes = [((2, 32, 24, 24), (32, 32, 3, 3), 1, 1), ((2, 64, 12, 12), (64, 64, 3, 3), 1, 1),
              ((2, 16, 24, 24), (32, 16, 1, 1), 2, 0)] * 6
    specs, xs = [], []
    for xs_, ws_, st, pad in shapes:
        xs.append(torch.randn(xs_, generator=g).to(DEV))
        specs.append((xs_, (torch.randn(ws_, generator=g) * 0.1).to(DEV), st, pad))
    for q in ("po2", "po2+"):
        ref = [_lib.qconv2d(x, w, None, st, pad, 1, 1, 4, q) for x, (_, w, st, pad) in zip(xs, specs)]
        pc = _lib.PackedConvs(specs, 4, q)
        pc.pack()
        for i, x in enumerate(xs):
            assert torch.equal(pc.conv(i, x), ref[i]), i
        with pytest.raises(_lib.Po2qError, match="planned for input"):
            pc.conv(0, xs[1])


ORACLE_SHAPES = [(1, 16, 12, 224), (2, 16, 9, 128), (1, 32, 10, 112), (2, 32, 7, 96), (1, 16, 5, 40)]


@pytest.mark.parametrize("shape", ORACLE_SHAPES, ids=[str(s) for s in ORACLE_SHAPES])
@pytest.mark.parametrize("mode", ["po2", "po2+"])
def test_s2ds_vs_oracle(shape, mode):
    """Both outputs of the fused stride-2 transition against the oracle (C restatement of the
    reference quantizer + fp64 conv): conv1 3x3 s2 p1 and downsample.0 1x1 s2 p0, each with its
    own Q(w) (reference models/resnet.py:55-71, :150-163)."""
    from oracle import oracle as O
    from tests._util import normwise_err

    N, C, H, W = shape
    x, w, wds = make(N, C, H, W, 31 + H + C)
    y, yds = _lib.qconv2d_s2ds(x, w, wds, 4, mode)
    xn = x.cpu().numpy()
    ref, _ = O.qconv2d(xn, w.cpu().numpy(), None, 2, 1, 1, 1, 4, mode)
    refds, _ = O.qconv2d(xn, wds.cpu().numpy(), None, 2, 0, 1, 1, 4, mode)
    assert normwise_err(y.cpu().numpy(), ref) <= CONV_TOL, normwise_err(y.cpu().numpy(), ref)
    assert normwise_err(yds.cpu().numpy(), refds) <= CONV_TOL, normwise_err(yds.cpu().numpy(), refds)


def test_s2ds_epilogues_vs_oracle():
    """Eval BN + ReLU on conv1 and eval BN on the shortcut, against the oracle."""
    import numpy as np

    from oracle import oracle as O
    from tests._util import normwise_err

    for C, W in ((16, 128), (32, 112)):
        x, w, wds = make(2, C, 8, W, 5 + C)
        g = torch.Generator().manual_seed(4)
        ps, psd = (torch.rand(2 * C, generator=g) + 0.5), (torch.rand(2 * C, generator=g) + 0.5)
        pb, pbd = (torch.randn(2 * C, generator=g) * 0.1), (torch.randn(2 * C, generator=g) * 0.1)
        y, yds = _lib.qconv2d_s2ds(x, w, wds, 4, "po2", post_scale=ps.to(DEV), post_shift=pb.to(DEV), act="relu",
                                   post_scale_ds=psd.to(DEV), post_shift_ds=pbd.to(DEV))
        v = lambda t: t.numpy().astype(np.float64).reshape(1, -1, 1, 1)  # noqa: E731
        xn = x.cpu().numpy()
        ref = np.maximum(O.qconv2d(xn, w.cpu().numpy(), None, 2, 1, 1, 1, 4, "po2")[0] * v(ps) + v(pb), 0.0)
        refds = O.qconv2d(xn, wds.cpu().numpy(), None, 2, 0, 1, 1, 4, "po2")[0] * v(psd) + v(pbd)
        assert normwise_err(y.cpu().numpy(), ref) <= CONV_TOL
        assert normwise_err(yds.cpu().numpy(), refds) <= CONV_TOL
