"""GPU parity of the small-image chain kernel (po2q_qconv2d_chain_f32, po2q_conv_chain.hip): n
quantized 3x3 / stride-1 C -> C convs in one launch, one block per image, against the oracle
layer by layer (O.qconv2d: fp64 accumulation on the bit-exact Q(w), each layer's output rounded to
fp32 as the reference's tensors are) and against the library's own per-layer path.

Tolerance: max|y - y_ref| <= 1e-5 max|y_ref| on the chain's output (CONV_TOL)."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from po2_quantization_amd import _lib
from tests._util import CONV_TOL, normwise_err

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
ACT_NP = {"none": lambda t: t, "relu": lambda t: np.maximum(t, 0.0), "relu6": lambda t: np.clip(t, 0.0, 6.0),
          "silu": lambda t: t / (1.0 + np.exp(-t))}


def oracle_chain(x, ws, mode, ps=None, pb=None, acts=None, res_from=None):
    """The reference's layer sequence on the oracle (resnet.py:55-71 order: conv, BN affine,
    + shortcut, activation), every intermediate an fp32 tensor.  Test-only checker."""
    a = [x.astype(np.float32)]
    for l, w in enumerate(ws):
        y, _ = O.qconv2d(a[l], w, None, 1, 1, 1, 1, 4, mode)
        if ps is not None and ps[l] is not None:
            y = y * ps[l].astype(np.float64).reshape(1, -1, 1, 1) + pb[l].astype(np.float64).reshape(1, -1, 1, 1)
        if res_from is not None and res_from[l] is not None and res_from[l] >= 0:
            y = y + a[res_from[l]].astype(np.float64)
        y = ACT_NP[acts[l] if acts else "none"](y)
        a.append(y.astype(np.float32) if l + 1 < len(ws) else y)
    return a[-1]


def make(N, C, H, W, n, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.relu(torch.randn(N, C, H, W, generator=g))
    ws = [torch.randn(C, C, 3, 3, generator=g) * (0.5 / np.sqrt(9 * C)) * 2 for _ in range(n)]
    return x, ws


CHAIN_SHAPES = [(3, 16, 32, 32, 5), (2, 32, 16, 16, 4), (2, 64, 8, 8, 3), (1, 16, 7, 12, 3), (2, 32, 5, 8, 2),
                (1, 64, 8, 16, 2), (2, 16, 1, 4, 3), (1, 16, 3, 36, 4)]


@pytest.mark.parametrize("shape", CHAIN_SHAPES, ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("mode", ["po2", "po2+"])
def test_chain_plain_vs_oracle(shape, mode):
    N, C, H, W, n = shape
    x, ws = make(N, C, H, W, n, seed=N * 100 + C + H + n)
    y = _lib.qconv2d_chain(x.to(DEV), [w.to(DEV) for w in ws], 4, mode)
    ref = oracle_chain(x.numpy(), [w.numpy() for w in ws], mode)
    err = normwise_err(y.cpu().numpy(), ref)
    assert err <= CONV_TOL, err


@pytest.mark.parametrize("shape", [(2, 16, 32, 32, 6), (2, 32, 16, 16, 5), (3, 64, 8, 8, 4), (1, 32, 9, 12, 4)],
                         ids=lambda s: "x".join(map(str, s)))
def test_chain_basic_blocks_vs_oracle(shape):
    """The BasicBlock form (resnet.py:55-71): conv1 -> BN -> ReLU, conv2 -> BN -> + block input ->
    ReLU, block after block (res_from = the block's first layer), plus a trailing odd layer with
    relu6 / silu to cover every activation."""
    N, C, H, W, n = shape
    x, ws = make(N, C, H, W, n, seed=7 + C + H)
    g = torch.Generator().manual_seed(3)
    ps = [torch.rand(C, generator=g) + 0.5 for _ in range(n)]
    pb = [torch.randn(C, generator=g) * 0.1 for _ in range(n)]
    acts = ["relu"] * n
    res = [-1 if l % 2 == 0 else l - 1 for l in range(n)]
    if n % 2:
        acts[-1] = "silu"
    else:
        acts[-1] = "relu6"
    y = _lib.qconv2d_chain(x.to(DEV), [w.to(DEV) for w in ws], 4, "po2", post_scales=[t.to(DEV) for t in ps],
                           post_shifts=[t.to(DEV) for t in pb], acts=acts, res_from=res)
    ref = oracle_chain(x.numpy(), [w.numpy() for w in ws], "po2", [t.numpy() for t in ps], [t.numpy() for t in pb],
                       acts, res)
    err = normwise_err(y.cpu().numpy(), ref)
    assert err <= CONV_TOL, err


def test_chain_long_residual_and_bias():
    """Residuals reaching back over two layers (the source held in registers across a layer that
    adds nothing), the network input as a source, conv biases, against the library's own
    per-layer fused calls."""
    N, C, H, W, n = 2, 32, 8, 16, 6
    x, ws = make(N, C, H, W, n, seed=11)
    g = torch.Generator().manual_seed(4)
    bs = [torch.randn(C, generator=g) * 0.1 if l % 2 else None for l in range(n)]
    res = [-1, -1, 0, -1, -1, 3]
    xd, wd = x.to(DEV), [w.to(DEV) for w in ws]
    bd = [b.to(DEV) if b is not None else None for b in bs]
    y = _lib.qconv2d_chain(xd, wd, 4, "po2", biases=bd, acts=["relu"] * n, res_from=res)
    a = [xd]
    for l in range(n):
        r = a[res[l]] if res[l] >= 0 else None
        a.append(_lib.qconv2d_fused(a[l], wd[l], bd[l], 1, 1, 1, 1, 4, "po2", residual=r, act="relu"))
    err = ((y - a[-1]).abs().max() / a[-1].abs().max()).item()
    assert err <= CONV_TOL, err


def test_chain_full_size_config2_stage1():
    """Config 2's stage-1 run at full size (bs = 256, 32x32, 18 layers) against the same layers run
    one launch each (the small-image / row kernels)."""
    torch.manual_seed(0)
    x = torch.relu(torch.randn(256, 16, 32, 32, device=DEV))
    ws = [torch.randn(16, 16, 3, 3, device=DEV) * 0.12 for _ in range(18)]
    y = _lib.qconv2d_chain(x, ws, 4, "po2")
    a = x
    for w in ws:
        a = _lib.qconv2d(a, w, None, 1, 1, 1, 1, 4, "po2")
    err = ((y - a).abs().max() / a.abs().max()).item()
    assert err <= CONV_TOL, err


def test_chain_nonfinite_inputs_match_oracle():
    """+-inf / NaN in the input propagate exactly as the oracle's fp64 direct conv has them."""
    x, ws = make(1, 16, 6, 8, 2, seed=5)
    x[0, 3, 2, 4] = float("inf")
    x[0, 7, 0, 0] = float("nan")
    y = _lib.qconv2d_chain(x.to(DEV), [w.to(DEV) for w in ws], 4, "po2").cpu().numpy()
    ref = oracle_chain(x.numpy(), [w.numpy() for w in ws], "po2")
    assert np.array_equal(np.isnan(y), np.isnan(ref))
    assert np.array_equal(np.isposinf(y), np.isposinf(ref)) and np.array_equal(np.isneginf(y), np.isneginf(ref))
    fin = np.isfinite(ref)
    assert np.abs(y[fin] - ref[fin]).max() <= CONV_TOL * np.abs(ref[fin]).max()


def test_chain_rejects():
    x = torch.randn(1, 48, 8, 8, device=DEV)
    with pytest.raises(_lib.Po2qError, match="C in"):
        _lib.qconv2d_chain(x, [torch.randn(48, 48, 3, 3, device=DEV)] * 2)
    x = torch.randn(1, 16, 8, 8, device=DEV)
    w = torch.randn(16, 16, 3, 3, device=DEV)
    with pytest.raises(_lib.Po2qError, match="res_from"):
        _lib.qconv2d_chain(x, [w, w], res_from=[-1, 2])
    with pytest.raises(_lib.Po2qError, match="one residual source at a time"):
        _lib.qconv2d_chain(x, [w] * 4, res_from=[-1, -1, 0, 1])
    with pytest.raises(_lib.Po2qError, match="must be"):
        _lib.qconv2d_chain(x, [w, torch.randn(16, 16, 1, 1, device=DEV)])
    with pytest.raises(_lib.Po2qError, match="mode"):
        _lib.qconv2d_chain(x, [w, w], mode="none")


def test_bench_chain_forward_equals_per_layer_forward():
    """bench.py's config-2 chain (ResNet56 @32: three chain launches + the stride-2 transitions)
    gives the per-layer forward's logits."""
    import bench

    c = bench.QConvChain(9, 10, "po2", 4, "auto", torch.device(DEV), seed=0)
    x = torch.relu(torch.randn(8, 16, 32, 32, generator=torch.Generator().manual_seed(1))).to(DEV)
    with torch.no_grad():
        y_chain = c.forward(x)
        assert len(c.chains) == 3 and [len(r) for r, _ in c.chains.values()] == [18, 17, 17]
        c.chain = False
        y_ref = c.forward(x)
    err = ((y_chain - y_ref).abs().max() / y_ref.abs().max()).item()
    assert err <= CONV_TOL, err


@pytest.mark.parametrize("shape", [(2, 32, 16, 16, 5), (3, 64, 8, 8, 4), (1, 32, 9, 12, 4), (2, 64, 8, 16, 3),
                                   (2, 32, 5, 8, 2)], ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("variant", ["8", "9"])
def test_chain_double_buffered_planes_vs_oracle(shape, variant, monkeypatch):
    """The default two plane sets (no barrier between a layer's MFMAs and its epilogue; C = 32 / 64)
    against the one-set kernel (PO2Q_CHAIN_VARIANT bit 3), exact-fit and checked forms, in the
    BasicBlock form: bit for bit, and within the bar of the oracle."""
    N, C, H, W, n = shape
    x, ws = make(N, C, H, W, n, seed=11 + C + H)
    g = torch.Generator().manual_seed(4)
    ps = [(torch.rand(C, generator=g) + 0.5).to(DEV) for _ in range(n)]
    pb = [(torch.randn(C, generator=g) * 0.1).to(DEV) for _ in range(n)]
    acts = ["relu"] * n
    res = [-1 if l % 2 == 0 else l - 1 for l in range(n)]
    xd, wd = x.to(DEV), [w.to(DEV) for w in ws]
    monkeypatch.setenv("PO2Q_CHAIN_VARIANT", variant)  # one set (variant 9: checked form too)
    ref1 = _lib.qconv2d_chain(xd, wd, 4, "po2", post_scales=ps, post_shifts=pb, acts=acts, res_from=res)
    monkeypatch.setenv("PO2Q_CHAIN_VARIANT", str(int(variant) - 8))
    y = _lib.qconv2d_chain(xd, wd, 4, "po2", post_scales=ps, post_shifts=pb, acts=acts, res_from=res)
    assert torch.equal(y, ref1)
    ref = oracle_chain(x.numpy(), [w.numpy() for w in ws], "po2", [t.cpu().numpy() for t in ps],
                       [t.cpu().numpy() for t in pb], acts, res)
    assert normwise_err(y.cpu().numpy(), ref) <= CONV_TOL
