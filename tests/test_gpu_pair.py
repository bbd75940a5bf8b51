"""GPU parity of the two-conv kernel (po2q_qconv2d_pair_f32): a ResNet56 stage-1 BasicBlock's
conv1 -> bn1 -> relu -> conv2 -> bn2 (+ shortcut) -> relu (reference models/resnet.py:55-71,
each conv QuantizedConv2d.forward, models/quantized_conv.py:32-38) in one launch, against the
same chain in torch fp32 on Q(w) (a plain PyTorch fp32 reference) and against two fused
single-conv calls.  Bar: normwise 1e-5 (CONV_TOL)."""
import pytest
import torch
import torch.nn.functional as F

from po2_quantization_amd import _lib
from tests._util import CONV_TOL

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
ACT = {"none": lambda t: t, "relu": torch.relu, "relu6": F.relu6, "silu": F.silu}


def nerr(y, ref):
    return ((y - ref).abs().max() / ref.abs().max()).item()


def make(N, H, W, seed, affine, C=16):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(N, C, H, W, generator=g).to(DEV)
    w1 = (torch.randn(C, C, 3, 3, generator=g) * 0.12).to(DEV)
    w2 = (torch.randn(C, C, 3, 3, generator=g) * 0.12).to(DEV)
    e = {}
    if affine:
        for k in ("post_scale1", "post_scale2"):
            e[k] = (torch.rand(C, generator=g) + 0.5).to(DEV)
        for k in ("post_shift1", "post_shift2"):
            e[k] = (torch.randn(C, generator=g) * 0.1).to(DEV)
    return x, w1, w2, e


def torch_chain(x, w1, w2, e, act1, act2, res, mode="po2", bias1=None, bias2=None):
    q1, q2 = _lib.quantize(w1, 4, mode), _lib.quantize(w2, 4, mode)
    h = F.conv2d(x, q1, bias1, 1, 1)
    if "post_scale1" in e:
        h = h * e["post_scale1"].view(1, -1, 1, 1) + e["post_shift1"].view(1, -1, 1, 1)
    h = ACT[act1](h)
    y = F.conv2d(h, q2, bias2, 1, 1)
    if "post_scale2" in e:
        y = y * e["post_scale2"].view(1, -1, 1, 1) + e["post_shift2"].view(1, -1, 1, 1)
    if res is not None:
        y = y + res
    return ACT[act2](y)


SHAPES = [(2, 20, 32, 16), (1, 9, 224, 16), (3, 37, 68, 16), (2, 1, 36, 16), (1, 2, 8, 16), (2, 56, 56, 16),
          (4, 17, 224, 16),
          (2, 20, 32, 32), (1, 9, 112, 32), (3, 37, 68, 32), (2, 1, 36, 32), (1, 2, 8, 32), (4, 13, 112, 32)]


@pytest.mark.parametrize("shape", SHAPES, ids=[str(s) for s in SHAPES])
@pytest.mark.parametrize("variant", ["20", "23", "123"])
def test_pair_chain_vs_torch(shape, variant, monkeypatch):
    monkeypatch.setenv("PO2Q_PAIR_VARIANT", variant)
    N, H, W, C = shape
    x, w1, w2, _ = make(N, H, W, hash(shape) & 0xFFFF, False, C)
    y = _lib.qconv2d_pair(x, w1, w2, 4, "po2")
    ref = torch_chain(x, w1, w2, {}, "none", "none", None)
    assert nerr(y, ref) <= CONV_TOL, nerr(y, ref)


@pytest.mark.parametrize("shape", [(2, 20, 32, 16), (2, 23, 224, 16), (3, 37, 68, 16), (2, 20, 32, 32),
                                   (2, 23, 112, 32), (2, 11, 160, 16), (1, 7, 200, 16)])
@pytest.mark.parametrize("acts,with_res", [(("relu", "relu"), True), (("relu", "relu"), False),
                                           (("relu6", "silu"), True), (("none", "relu"), True)])
def test_pair_block_epilogue_vs_torch(shape, acts, with_res):
    """act2(bn2(conv2(act1(bn1(conv1 x)))) + x): the BasicBlock with its identity shortcut."""
    N, H, W, C = shape
    x, w1, w2, e = make(N, H, W, 11 + H, True, C)
    g = torch.Generator().manual_seed(5)
    b1 = (torch.randn(C, generator=g) * 0.1).to(DEV)
    y = _lib.qconv2d_pair(x, w1, w2, 4, "po2+", bias1=b1, act1=acts[0], act2=acts[1],
                          residual=x if with_res else None, **e)
    ref = torch_chain(x, w1, w2, e, acts[0], acts[1], x if with_res else None, "po2+", bias1=b1)
    assert nerr(y, ref) <= CONV_TOL, nerr(y, ref)


@pytest.mark.parametrize("C,W", [(16, 224), (32, 112)])
def test_pair_equals_two_fused_calls(C, W):
    """The same result as qconv2d_fused twice (its row kernel: same bf16x3 arithmetic)."""
    x, w1, w2, e = make(4, 40, W, 3, True, C)
    y = _lib.qconv2d_pair(x, w1, w2, 4, "po2", act1="relu", act2="relu", residual=x, **e)
    h = _lib.qconv2d_fused(x, w1, None, 1, 1, 1, 1, 4, "po2", post_scale=e["post_scale1"],
                           post_shift=e["post_shift1"], act="relu")
    y2 = _lib.qconv2d_fused(h, w2, None, 1, 1, 1, 1, 4, "po2", post_scale=e["post_scale2"],
                            post_shift=e["post_shift2"], residual=x, act="relu")
    assert nerr(y, y2) <= 1e-6, nerr(y, y2)


@pytest.mark.parametrize("C,H", [(16, 224), (32, 112)])
def test_pair_full_size(C, H):
    """BASELINE size (bs = 256 @224: stage 1, and stage 2 @112) at the bench's exact launch geometry:
    against torch's fp32 chain on every image, and against the fp64 oracle (oracle/oracle.py qconv2d,
    conv1 then conv2 on its output) on sampled images -- the first and last block of the grid, and
    images whose blocks land on different XCDs of the remapped grid."""
    from oracle import oracle as O

    torch.manual_seed(0)
    x = torch.relu(torch.randn(256, C, H, H, device=DEV))
    w1 = torch.randn(C, C, 3, 3, device=DEV) * (0.12 if C == 16 else 0.08)
    w2 = torch.randn(C, C, 3, 3, device=DEV) * (0.12 if C == 16 else 0.08)
    y = _lib.qconv2d_pair(x, w1, w2, 4, "po2")
    ref = torch_chain(x, w1, w2, {}, "none", "none", None)
    assert nerr(y, ref) <= CONV_TOL, nerr(y, ref)
    idx = [0, 37, 130, 255]
    xs = x[idx].cpu().numpy()
    h, _ = O.qconv2d(xs, w1.cpu().numpy(), None, 1, 1, 1, 1, 4, "po2")
    o, _ = O.qconv2d(h.astype("float32"), w2.cpu().numpy(), None, 1, 1, 1, 1, 4, "po2")
    ys = y[idx].cpu().numpy().astype("float64")
    err = abs(ys - o).max() / abs(o).max()
    assert err <= CONV_TOL, err


def test_pair_rejects():
    x = torch.randn(1, 64, 8, 8, device=DEV)
    w = torch.randn(64, 64, 3, 3, device=DEV)
    assert not _lib.pair_supported(x.shape)
    assert _lib.pair_supported((256, 16, 224, 224)) and not _lib.pair_supported((256, 16, 32, 32))
    assert _lib.pair_supported((256, 32, 112, 112))  # stage 2 @112: advised since round 3
    assert not _lib.pair_supported((256, 32, 16, 16))  # CIFAR stage 2: two single-conv launches (or the chain)
    with pytest.raises(_lib.Po2qError, match="16 or 32 channels"):
        _lib.qconv2d_pair(x, w, w)
    x = torch.randn(1, 16, 8, 10, device=DEV)
    w = torch.randn(16, 16, 3, 3, device=DEV)
    with pytest.raises(_lib.Po2qError, match="multiple of 4"):
        _lib.qconv2d_pair(x, w, w)
    with pytest.raises(_lib.Po2qError, match="mode"):
        _lib.qconv2d_pair(torch.randn(1, 16, 8, 8, device=DEV), w, w, mode="none")


def oracle_block(x, w1, w2, mode, e, act1, act2, res, bias1=None):
    """The reference BasicBlock chain (models/resnet.py:55-71) on the oracle: O.qconv2d (fp64
    accumulation on the bit-exact Q(w)) -> numpy affine / activation -> O.qconv2d -> + residual ->
    activation.  Test-only checker."""
    import numpy as np

    from oracle import oracle as O

    acts = {"none": lambda t: t, "relu": lambda t: np.maximum(t, 0.0),
            "relu6": lambda t: np.clip(t, 0.0, 6.0), "silu": lambda t: t / (1.0 + np.exp(-t))}
    v = lambda k: e[k].cpu().numpy().astype(np.float64).reshape(1, -1, 1, 1)  # noqa: E731
    h, _ = O.qconv2d(x.cpu().numpy(), w1.cpu().numpy(), None if bias1 is None else bias1.cpu().numpy(),
                     1, 1, 1, 1, 4, mode)
    if "post_scale1" in e:
        h = h * v("post_scale1") + v("post_shift1")
    h = acts[act1](h).astype(np.float32)  # the intermediate is an fp32 tensor in the reference
    y, _ = O.qconv2d(h, w2.cpu().numpy(), None, 1, 1, 1, 1, 4, mode)
    if "post_scale2" in e:
        y = y * v("post_scale2") + v("post_shift2")
    if res is not None:
        y = y + res.cpu().numpy().astype(np.float64)
    return acts[act2](y)


ORACLE_SHAPES = [(1, 9, 224, 16), (2, 12, 128, 16), (1, 10, 68, 16), (2, 7, 112, 32), (1, 11, 64, 32)]


@pytest.mark.parametrize("shape", ORACLE_SHAPES, ids=[str(s) for s in ORACLE_SHAPES])
@pytest.mark.parametrize("mode", ["po2", "po2+"])
def test_pair_vs_oracle(shape, mode):
    """conv_pair against the oracle (C restatement of the reference quantizer + fp64 conv), the
    plain chain: max|y - y_oracle| <= 1e-5 max|y_oracle|."""
    from tests._util import normwise_err

    N, H, W, C = shape
    x, w1, w2, _ = make(N, H, W, 101 + H, False, C)
    y = _lib.qconv2d_pair(x, w1, w2, 4, mode)
    ref = oracle_block(x, w1, w2, mode, {}, "none", "none", None)
    assert normwise_err(y.cpu().numpy(), ref) <= CONV_TOL, normwise_err(y.cpu().numpy(), ref)


@pytest.mark.parametrize("C,W", [(16, 224), (16, 96 + 32), (32, 112), (32, 64)])
def test_pair_block_vs_oracle(C, W):
    """The BasicBlock form BasicBlock.forward uses (E = 2: folded affine, compile-time ReLU): BN affine + ReLU, conv 2,
    BN affine, + identity shortcut, ReLU, against the oracle chain."""
    from tests._util import normwise_err

    x, w1, w2, e = make(2, 9, W, 7 + W, True, C)
    g = torch.Generator().manual_seed(9)
    b1 = (torch.randn(C, generator=g) * 0.1).to(DEV)
    for mode in ("po2", "po2+"):
        y = _lib.qconv2d_pair(x, w1, w2, 4, mode, bias1=b1, act1="relu", act2="relu", residual=x, **e)
        ref = oracle_block(x, w1, w2, mode, e, "relu", "relu", x, bias1=b1)
        assert normwise_err(y.cpu().numpy(), ref) <= CONV_TOL, (mode, normwise_err(y.cpu().numpy(), ref))


@pytest.mark.parametrize("pd", [5])
@pytest.mark.parametrize("shape", [(2, 23, 224, 16), (1, 224, 224, 16), (3, 9, 200, 16), (2, 31, 208, 16)])
def test_pair_memory_wave_bitwise_equal(pd, shape, monkeypatch):
    """The memory-wave kernel (PO2Q_PAIR_MW = ring slots: an eighth wave issues every x DMA, the
    compute waves issue none) moves the loads, not the arithmetic: bit for bit the one-role kernel's
    output (PO2Q_PAIR_MW=0: every compute wave DMAs its own share of the x rows; at C = 16 the
    default is the memory wave itself), plain and with the general (BN + activation) epilogue; and
    within the bar of torch's fp32 chain on Q(w)."""
    N, H, W, C = shape
    x, w1, w2, e = make(N, H, W, 41 + pd, True, C)
    forms = [{}, dict(act1="relu", act2="relu6", **e)]
    if C == 16:  # the identity residual read from the x ring (BasicBlock form and the general epilogue)
        forms += [dict(act1="relu", act2="relu", residual=x, **e), dict(act1="relu6", act2="silu", residual=x, **e)]
    outs = []
    for kw in forms:
        monkeypatch.setenv("PO2Q_PAIR_MW", "0")
        ref = _lib.qconv2d_pair(x, w1, w2, 4, "po2", **kw)
        monkeypatch.setenv("PO2Q_PAIR_MW", str(pd))
        y = _lib.qconv2d_pair(x, w1, w2, 4, "po2", **kw)
        assert torch.equal(y, ref), (pd, shape, sorted(kw))
        outs.append(y)
    t = torch_chain(x, w1, w2, e, "relu", "relu6", None)  # forms[1]
    assert nerr(outs[1], t) <= CONV_TOL
    if C == 16 and W > 192 and pd == 5:  # 7-wave widths: with PO2Q_PAIR_MW unset the default is the
        monkeypatch.delenv("PO2Q_PAIR_MW", raising=False)  # role-split kernel without a residual, MW with one
        assert torch.equal(_lib.qconv2d_pair(x, w1, w2, 4, "po2"), outs[0])
        assert torch.equal(_lib.qconv2d_pair(x, w1, w2, 4, "po2", **forms[2]), outs[2])


@pytest.mark.parametrize("shape", [(2, 23, 224), (1, 224, 224), (3, 9, 200), (2, 1, 208), (4, 40, 224),
                                   (1, 2, 196)])
def test_pair_role_split_bitwise_equal_memory_wave(shape, monkeypatch):
    """Stage 1's role-split pair (conv_pair_rs16: seven conv-1 waves DMA and split x and write the
    intermediate ring, seven conv-2 waves read it two rows behind; the default at C = 16, W > 192
    without a residual) runs the memory-wave kernel's fragments, MFMA order and epilogue expressions,
    so its output is that kernel's bit for bit (PO2Q_PAIR_RS=0), plain and with the general epilogue;
    ragged heights, 1- and 2-row images and the narrowest 7-strip width included."""
    N, H, W = shape
    x, w1, w2, e = make(N, H, W, 61 + H + W, True, 16)
    g = torch.Generator().manual_seed(H * W)
    b1, b2 = (torch.randn(16, generator=g) * 0.1).to(DEV), (torch.randn(16, generator=g) * 0.1).to(DEV)
    forms = [{}, dict(act1="relu", act2="relu6", **e), dict(act1="silu", act2="relu", bias1=b1, bias2=b2, **e)]
    for mode in ("po2", "po2+"):
        for kw in forms:
            monkeypatch.setenv("PO2Q_PAIR_RS", "0")
            ref = _lib.qconv2d_pair(x, w1, w2, 4, mode, **kw)
            monkeypatch.delenv("PO2Q_PAIR_RS")
            y = _lib.qconv2d_pair(x, w1, w2, 4, mode, **kw)
            assert torch.equal(y, ref), (shape, mode, sorted(kw), nerr(y, ref))
    t = torch_chain(x, w1, w2, e, "relu", "relu6", None)
    assert nerr(_lib.qconv2d_pair(x, w1, w2, 4, "po2", **forms[1]), t) <= CONV_TOL


@pytest.mark.parametrize("shape", [(2, 23, 112, 32), (1, 112, 112, 32), (3, 9, 100, 32), (2, 1, 104, 32),
                                   (4, 13, 108, 32)])
def test_pair_w32_bitwise_equal_7wave_kernel(shape, monkeypatch):
    """Stage 2's 4-wave kernel (po2q_conv_pairw.hip: 32 columns per wave, both convs' weights in VGPRs,
    whole-line stores; the default for C = 32 at 96 < W <= 128) runs the 7-wave conv_pair<32>'s
    arithmetic -- the same fragments, the same MFMA order per accumulator, the same epilogue expressions
    -- so its output is bit for bit the 7-wave kernel's (PO2Q_PAIR_W32=0) in the plain, general and
    BasicBlock forms; ragged widths and 1-row images included."""
    N, H, W, C = shape
    x, w1, w2, e = make(N, H, W, 51 + W + H, True, C)
    g = torch.Generator().manual_seed(W)
    b1, b2 = (torch.randn(C, generator=g) * 0.1).to(DEV), (torch.randn(C, generator=g) * 0.1).to(DEV)
    forms = [{}, dict(act1="relu", act2="relu6", **e), dict(act1="relu", act2="relu", residual=x, **e),
             dict(act1="silu", act2="relu", residual=x.flip(3).contiguous(), bias1=b1, bias2=b2, **e)]
    for kw in forms:
        monkeypatch.setenv("PO2Q_PAIR_W32", "0")
        ref = _lib.qconv2d_pair(x, w1, w2, 4, "po2+", **kw)
        monkeypatch.setenv("PO2Q_PAIR_W32", "1")
        y = _lib.qconv2d_pair(x, w1, w2, 4, "po2+", **kw)
        assert torch.equal(y, ref), (shape, sorted(kw), nerr(y, ref))
    t = torch_chain(x, w1, w2, e, "relu", "relu", x, "po2+")
    monkeypatch.delenv("PO2Q_PAIR_W32", raising=False)
    assert nerr(_lib.qconv2d_pair(x, w1, w2, 4, "po2+", **forms[2]), t) <= CONV_TOL
