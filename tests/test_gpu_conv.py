"""GPU parity: fused quantize+conv (libpo2q) vs the reference golden vectors and
the oracle (fp64 direct conv of the bit-exact quantized weight).

Tolerance (BASELINE.md parity contract): max|y - y_ref| <= 1e-5 * max|y_ref|
per output tensor (normwise relative, fp32 arithmetic; ties of round() follow
torch.round = half-to-even, reproduced bit-exactly by the quantizer)."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from po2_quantization_amd import _lib
from po2_quantization_amd.models.quantized_conv import QuantizedConv2d
from po2_quantization_amd.utils.quantizers import quantizer_dict
from tests._util import CONV_TOL, load_json, load_npz, normwise_err

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
PRECISIONS = ["auto", "fp32", "bf16x3"]


def eligible_x3(mode, groups, bits=4):
    return mode != "none" and groups == 1 and bits <= 7


def run_native(x, w, b, stride, pad, dil, groups, bits, mode, precision="auto"):
    xt = torch.from_numpy(np.ascontiguousarray(x)).to(DEV)
    wt = torch.from_numpy(np.ascontiguousarray(w)).to(DEV)
    bt = torch.from_numpy(np.ascontiguousarray(b)).to(DEV) if b is not None else None
    return _lib.qconv2d(xt, wt, bt, stride, pad, dil, groups, bits, mode, 1, precision).cpu().numpy()


@pytest.mark.parametrize("precision", PRECISIONS)
def test_golden_conv_vectors(precision):
    d = load_npz("conv_kat.npz")
    for m in load_json("conv_kat.json"):
        n = m["name"]
        if precision == "bf16x3" and not eligible_x3(m["mode"], m["groups"], m["bits"]):
            continue
        b = d["b/" + n] if m["bias"] else None
        y = run_native(d["x/" + n], d["w/" + n], b, m["stride"], m["pad"], m["dil"], m["groups"],
                       m["bits"], m["mode"], precision)
        assert y.shape == d["y/" + n].shape, n
        assert normwise_err(y, d["y/" + n]) <= CONV_TOL, (n, normwise_err(y, d["y/" + n]))
        assert normwise_err(y, d["y64/" + n]) <= CONV_TOL, n


def test_golden_vectors_through_module():
    """Same vectors through the drop-in nn.Module (ctor defaults, bias param)."""
    d = load_npz("conv_kat.npz")
    for m in load_json("conv_kat.json"):
        n = m["name"]
        qfn = None if m["mode"] == "none" else quantizer_dict[m["mode"]]
        C, K = m["C"], m["K"]
        mod = QuantizedConv2d(C, K, (m["R"], m["S"]), stride=m["stride"], padding=m["pad"], dilation=m["dil"],
                              groups=m["groups"], bias=m["bias"], quantize_fn=qfn, bits=m["bits"]).to(DEV)
        with torch.no_grad():
            mod.weight.copy_(torch.from_numpy(d["w/" + n]))
            if m["bias"]:
                mod.bias.copy_(torch.from_numpy(d["b/" + n]))
            y = mod(torch.from_numpy(d["x/" + n]).to(DEV)).cpu().numpy()
        assert normwise_err(y, d["y/" + n]) <= CONV_TOL, n


# ResNet56 / MobileNet conv kinds at reduced batch & spatial size vs the oracle
SHAPES = [
    # N, C, H, W, K, R, S, stride, pad, dil, groups
    (2, 16, 40, 36, 16, 3, 3, 1, 1, 1, 1),
    (2, 32, 20, 20, 32, 3, 3, 1, 1, 1, 1),
    (1, 64, 14, 14, 64, 3, 3, 1, 1, 1, 1),
    (2, 16, 33, 31, 32, 3, 3, 2, 1, 1, 1),
    (2, 32, 16, 16, 64, 3, 3, 2, 1, 1, 1),
    (2, 16, 32, 32, 32, 1, 1, 2, 0, 1, 1),
    (2, 32, 16, 16, 64, 1, 1, 2, 0, 1, 1),
    (2, 3, 32, 32, 16, 3, 3, 1, 1, 1, 1),
    (2, 160, 4, 4, 960, 1, 1, 1, 0, 1, 1),
    (2, 960, 2, 2, 160, 1, 1, 1, 0, 1, 1),
    (2, 144, 8, 8, 144, 3, 3, 2, 1, 1, 144),
    (2, 48, 9, 9, 24, 3, 3, 1, 1, 1, 1),
    (1, 20, 13, 11, 36, 3, 3, 1, 2, 2, 2),
    (1, 8, 70, 70, 24, 3, 3, 1, 1, 1, 1),
    (3, 16, 8, 8, 16, 3, 3, 1, 1, 1, 1),
    (1, 12, 9, 9, 20, 5, 3, 2, (2, 1), 1, 4),
    # row-streaming kernel edges: strip wider than the image, ragged last strip /
    # segment, C = 32 -> K = 16, one-row images
    (2, 16, 5, 4, 16, 3, 3, 1, 1, 1, 1),
    (1, 16, 37, 68, 16, 3, 3, 1, 1, 1, 1),
    (1, 32, 23, 20, 16, 3, 3, 1, 1, 1, 1),
    (2, 32, 1, 12, 32, 3, 3, 1, 1, 1, 1),
    # full-row blocks (C = K = 16): one-row image, seven waves with a ragged last strip
    (2, 16, 1, 36, 16, 3, 3, 1, 1, 1, 1),
    (1, 16, 9, 220, 16, 3, 3, 1, 1, 1, 1),
    # C = K = 64 (output channels across a block's waves): ragged strip, short segment
    (2, 64, 12, 40, 64, 3, 3, 1, 1, 1, 1),
    (1, 64, 3, 8, 64, 3, 3, 1, 1, 1, 1),
    # stride-2 full-row kernel (16 -> 32): two waves with a ragged strip, odd rows, one wave
    # with one DMA per row, a wide image
    (2, 16, 40, 40, 32, 3, 3, 2, 1, 1, 1),
    (1, 16, 9, 64, 32, 3, 3, 2, 1, 1, 1),
    (1, 16, 17, 8, 32, 3, 3, 2, 1, 1, 1),
    (2, 16, 30, 224, 32, 3, 3, 2, 1, 1, 1),
    (2, 32, 40, 40, 64, 3, 3, 2, 1, 1, 1),   # the same kernel, 32 -> 64
    (1, 32, 17, 8, 64, 3, 3, 2, 1, 1, 1),
    (2, 32, 30, 112, 64, 3, 3, 2, 1, 1, 1),
]


@pytest.mark.parametrize("shape", SHAPES, ids=[str(s) for s in SHAPES])
@pytest.mark.parametrize("mode", ["po2", "po2+", "none"])
@pytest.mark.parametrize("precision", PRECISIONS)
def test_shapes_vs_oracle(shape, mode, precision):
    N, C, H, W, K, R, S, st, pad, dil, groups = shape
    g = torch.Generator().manual_seed(hash(shape) & 0xFFFF)
    x = torch.randn(N, C, H, W, generator=g).numpy()
    w = (torch.randn(K, C // groups, R, S, generator=g) * 0.2).numpy()
    b = (torch.randn(K, generator=g) * 0.1).numpy() if K % 3 == 0 else None
    if precision == "bf16x3" and not eligible_x3(mode, groups):
        with pytest.raises(RuntimeError, match="bf16x3"):
            run_native(x, w, b, st, pad, dil, groups, 4, mode, precision)
        return
    y = run_native(x, w, b, st, pad, dil, groups, 4, mode, precision)
    ref, _ = O.qconv2d(x, w, b, st, pad, dil, groups, 4, mode)
    assert y.shape == ref.shape
    assert normwise_err(y, ref) <= CONV_TOL, normwise_err(y, ref)


FULL_LAYERS = [  # BASELINE config (bs=256, 224x224): every distinct ResNet56 qconv shape
    (16, 224, 16, 3, 1, 1), (16, 224, 32, 3, 2, 1), (16, 224, 32, 1, 2, 0), (32, 112, 32, 3, 1, 1),
    (32, 112, 64, 3, 2, 1), (32, 112, 64, 1, 2, 0), (64, 56, 64, 3, 1, 1),
]


@pytest.mark.parametrize("layer", FULL_LAYERS, ids=[str(l) for l in FULL_LAYERS])
def test_full_size_resnet56_layers_vs_torch_fp32(layer):
    """BASELINE size (bs=256, 224x224 input): against torch's own fp32 GPU conv of
    the bit-exact quantized weight (a plain PyTorch fp32 reference of the same op)."""
    C, H, K, R, st, pad = layer
    torch.manual_seed(0)
    x = torch.randn(256, C, H, H, device=DEV)
    w = torch.randn(K, C, R, R, device=DEV) * 0.1
    y = _lib.qconv2d(x, w, None, st, pad, 1, 1, 4, "po2")
    qw = _lib.quantize(w, 4, "po2")
    ref = torch.nn.functional.conv2d(x, qw, None, st, pad)
    err = ((y - ref).abs().max() / ref.abs().max()).item()
    assert err <= CONV_TOL, err
    # spot-check images at both ends of the batch against the fp64 oracle as well
    idx = [0, 255]
    o, _ = O.qconv2d(x[idx].cpu().numpy(), w.cpu().numpy(), None, st, pad, 1, 1, 4, "po2")
    assert normwise_err(y[idx].cpu().numpy(), o) <= CONV_TOL


PLAN_SHAPES = [s for s in SHAPES if s[-1] == 1]


@pytest.mark.parametrize("shape", PLAN_SHAPES, ids=[str(s) for s in PLAN_SHAPES])
def test_every_candidate_plan_vs_oracle(shape):
    """Autotuning may select any candidate plan, so each one must meet the parity bar."""
    N, C, H, W, K, R, S, st, pad, dil, groups = shape
    g = torch.Generator().manual_seed(hash(shape) & 0xFFFF)
    x = torch.randn(N, C, H, W, generator=g)
    w = torch.randn(K, C // groups, R, S, generator=g) * 0.2
    b = torch.randn(K, generator=g) * 0.1
    ref, _ = O.qconv2d(x.numpy(), w.numpy(), b.numpy(), st, pad, dil, groups, 4, "po2+")
    plans = _lib.plans(N, C, H, W, K, R, S, st, pad, dil, groups, 4, "po2+")
    xd, wd, bd = x.to(DEV), w.to(DEV), b.to(DEV)
    for i, desc in enumerate(plans):
        y = _lib.qconv2d(xd, wd, bd, st, pad, dil, groups, 4, "po2+", plan=i).cpu().numpy()
        assert normwise_err(y, ref) <= CONV_TOL, (desc, normwise_err(y, ref))


@pytest.mark.parametrize("layer", FULL_LAYERS, ids=[str(l) for l in FULL_LAYERS])
def test_full_size_every_candidate_plan(layer):
    """BASELINE-size layers through every candidate plan vs torch fp32 conv of Q(w)."""
    C, H, K, R, st, pad = layer
    torch.manual_seed(1)
    x = torch.randn(256, C, H, H, device=DEV)
    w = torch.randn(K, C, R, R, device=DEV) * 0.1
    ref = torch.nn.functional.conv2d(x, _lib.quantize(w, 4, "po2"), None, st, pad)
    amax = ref.abs().max()
    for i, desc in enumerate(_lib.plans(256, C, H, H, K, R, R, st, pad)):
        y = _lib.qconv2d(x, w, None, st, pad, 1, 1, 4, "po2", plan=i)
        err = ((y - ref).abs().max() / amax).item()
        assert err <= CONV_TOL, (desc, err)
        del y


def test_autotune_picks_a_candidate_and_keeps_parity(monkeypatch):
    """benchmark mode (cudnn.benchmark counterpart): the first call times every
    candidate, later calls and describe() use the winner; results stay in parity."""
    monkeypatch.setattr(_lib, "benchmark", True)
    shape = (2, 16, 40, 36, 32, 3, 3, 1, 1, 1, 1)
    N, C, H, W, K, R, S, st, pad, dil, groups = shape
    g = torch.Generator().manual_seed(7)
    x = torch.randn(N, C, H, W, generator=g)
    w = torch.randn(K, C, R, S, generator=g) * 0.2
    ref, _ = O.qconv2d(x.numpy(), w.numpy(), None, st, pad, dil, groups, 4, "po2")
    plans = _lib.plans(N, C, H, W, K, R, S, st, pad, dil, groups, 4, "po2")
    y1 = _lib.qconv2d(x.to(DEV), w.to(DEV), None, st, pad, dil, groups, 4, "po2").cpu().numpy()
    assert normwise_err(y1, ref) <= CONV_TOL
    chosen = _lib.describe(N, C, H, W, K, R, S, st, pad, dil, groups, 4, "po2")
    assert chosen in plans
    y2 = _lib.qconv2d(x.to(DEV), w.to(DEV), None, st, pad, dil, groups, 4, "po2").cpu().numpy()
    assert np.array_equal(y1, y2)
    # graph capture never autotunes (the sweep synchronises): a fresh shape is planned heuristically
    with pytest.raises(RuntimeError, match="graph capture"):
        L = _lib.load()
        xs, ws_ = x.to(DEV), w.to(DEV)
        y = torch.empty(N, K, H, W, device=DEV)
        ws = torch.empty(1 << 20, dtype=torch.uint8, device=DEV)
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            st_ = L.po2q_qconv2d_autotune(xs.data_ptr(), ws_.data_ptr(), None, y.data_ptr(), N, C, H, W, K, R, S,
                                          1, 1, 1, 1, 1, 1, 1, 4, 1, 1, 0, ws.data_ptr(), ws.numel(),
                                          torch.cuda.current_stream().cuda_stream, None, 0)
        _lib._check(st_)


def test_backward_matches_torch_ste():
    torch.manual_seed(1)
    x = torch.randn(4, 16, 12, 12, device=DEV, requires_grad=True)
    mod = QuantizedConv2d(16, 32, 3, stride=2, bias=True, quantize_fn=quantizer_dict["po2"], bits=4).to(DEV)
    y = mod(x)
    gy = torch.randn_like(y)
    y.backward(gy)
    x2 = x.detach().clone().requires_grad_(True)
    w2 = mod.weight.detach().clone().requires_grad_(True)
    b2 = mod.bias.detach().clone().requires_grad_(True)
    qw = w2 + (_lib.quantize(w2.detach(), 4, "po2") - w2).detach()  # STE
    y2 = torch.nn.functional.conv2d(x2, qw, b2, 2, 1)
    y2.backward(gy)
    assert torch.allclose(y, y2, rtol=1e-4, atol=1e-5)
    assert torch.allclose(x.grad, x2.grad, rtol=1e-4, atol=1e-5)
    assert torch.allclose(mod.weight.grad, w2.grad, rtol=1e-4, atol=1e-4)
    assert torch.allclose(mod.bias.grad, b2.grad, rtol=1e-4, atol=1e-4)


def test_errors_match_reference_behaviour():
    x = torch.randn(1, 5, 8, 8, device=DEV)
    with pytest.raises(RuntimeError, match="channels"):
        _lib.qconv2d(x, torch.randn(4, 4, 3, 3, device=DEV), None, 1, 1, 1, 1, 4, "po2")
    with pytest.raises(RuntimeError, match="kernel size"):
        _lib.qconv2d(torch.randn(1, 4, 2, 2, device=DEV), torch.randn(4, 4, 5, 5, device=DEV), None,
                     1, 0, 1, 1, 4, "po2")
    with pytest.raises(RuntimeError, match="float32"):
        _lib.qconv2d(x.double(), torch.randn(4, 5, 3, 3, device=DEV), None, 1, 1, 1, 1, 4, "po2")


def test_weight_special_values():
    """all-zero weights -> NaN output (0/0 in the reference quantizer); NaN weight -> NaN."""
    x = torch.randn(1, 4, 6, 6, device=DEV)
    y = _lib.qconv2d(x, torch.zeros(4, 4, 3, 3, device=DEV), None, 1, 1, 1, 1, 4, "po2")
    assert torch.isnan(y).all()
    w = torch.randn(4, 4, 3, 3, device=DEV)
    w[0, 0, 0, 0] = float("nan")
    assert torch.isnan(_lib.qconv2d(x, w, None, 1, 1, 1, 1, 4, "po2+")).all()


FUSED_SHAPES = [  # (N, C, H, W, K, R, stride, pad, groups): row kernels, K-split, tile, depthwise, 1x1
    (2, 16, 40, 36, 16, 3, 1, 1, 1),
    (2, 32, 20, 24, 32, 3, 1, 1, 1),
    (1, 64, 12, 40, 64, 3, 1, 1, 1),
    (2, 16, 33, 31, 32, 3, 2, 1, 1),
    (2, 32, 16, 16, 64, 1, 2, 0, 1),
    (2, 96, 9, 9, 96, 3, 1, 1, 96),
    (2, 16, 40, 40, 32, 3, 2, 1, 1),
]


@pytest.mark.parametrize("shape", FUSED_SHAPES, ids=[str(s) for s in FUSED_SHAPES])
@pytest.mark.parametrize("act", ["none", "relu", "relu6", "silu"])
@pytest.mark.parametrize("with_res", [False, True])
def test_fused_epilogue_vs_torch(shape, act, with_res):
    """po2q_qconv2d_fused_f32 == act(bn_eval(F.conv2d(x, Q(w))) + residual) in torch fp32
    (the reference's block order, resnet.py:55-71 / mobilenet.py:32-33 / mobile_vit.py:20-21)."""
    N, C, H, W, K, R, st, pad, groups = shape
    g = torch.Generator().manual_seed(hash((shape, act, with_res)) & 0xFFFF)
    x = torch.randn(N, C, H, W, generator=g).to(DEV)
    w = (torch.randn(K, C // groups, R, R, generator=g) * 0.2).to(DEV)
    bn = torch.nn.BatchNorm2d(K).to(DEV).eval()
    with torch.no_grad():
        bn.weight.copy_(1.0 + 0.2 * torch.randn(K, generator=g))
        bn.bias.copy_(0.1 * torch.randn(K, generator=g))
        bn.running_mean.copy_(0.1 * torch.randn(K, generator=g))
        bn.running_var.copy_(torch.rand(K, generator=g) + 0.5)
    from po2_quantization_amd.models.quantized_conv import fold_bn

    acts = {"none": lambda t: t, "relu": torch.relu, "relu6": torch.nn.functional.relu6,
            "silu": torch.nn.functional.silu}
    with torch.no_grad():
        qw = _lib.quantize(w, 4, "po2")
        y0 = bn(torch.nn.functional.conv2d(x, qw, None, st, pad, 1, groups))
        res = torch.randn(y0.shape, generator=g).to(DEV) if with_res else None
        ref = acts[act](y0 + res if with_res else y0)
        ps, pb = fold_bn(bn)
        y = _lib.qconv2d_fused(x, w, None, st, pad, 1, groups, 4, "po2", post_scale=ps, post_shift=pb,
                               residual=res, act=act)
    err = ((y - ref).abs().max() / ref.abs().max()).item()
    assert err <= CONV_TOL, err


def test_fused_every_row_plan_and_rejects_bad_act():
    """Every candidate plan of a row-kernel shape gives the same fused result (the tuned
    plan is the one the fused entry runs); an unknown activation raises."""
    N, C, H, W, K = 1, 32, 16, 32, 32
    torch.manual_seed(3)
    x = torch.randn(N, C, H, W, device=DEV)
    w = torch.randn(K, C, 3, 3, device=DEV) * 0.1
    ps = torch.rand(K, device=DEV) + 0.5
    pb = torch.randn(K, device=DEV) * 0.1
    ref = torch.relu(_lib.qconv2d(x, w, None, 1, 1) * ps.view(1, -1, 1, 1) + pb.view(1, -1, 1, 1))
    y = _lib.qconv2d_fused(x, w, None, 1, 1, post_scale=ps, post_shift=pb, act="relu")
    assert ((y - ref).abs().max() / ref.abs().max()).item() <= CONV_TOL
    L = _lib.load()
    with pytest.raises(_lib.Po2qError, match="activation"):
        _lib._check(L.po2q_qconv2d_fused_f32(x.data_ptr(), w.data_ptr(), None, y.data_ptr(), N, C, H, W, K, 3, 3,
                                             1, 1, 1, 1, 1, 1, 1, 4, 1, 1, 0, None, None, None, 9,
                                             x.data_ptr(), 1 << 20, None))


def test_empty_batch_like_torch():
    """F.conv2d on an empty batch returns an empty [0, K, P, Q] output (quantized_conv.py:36)."""
    w = torch.randn(8, 4, 3, 3, device=DEV)
    y = _lib.qconv2d(torch.empty(0, 4, 9, 9, device=DEV), w, None, 2, 1)
    assert y.shape == (0, 8, 5, 5)
    y = _lib.qconv2d_fused(torch.empty(0, 4, 9, 9, device=DEV), w, None, 1, 1, act="relu")
    assert y.shape == (0, 8, 9, 9)


@pytest.mark.parametrize("shape", [(2, 16, 20, 32, 16), (1, 32, 13, 36, 32), (1, 64, 9, 40, 64)],
                         ids=["c16", "c32", "c64"])
def test_fused_epilogue_every_candidate_plan(shape, monkeypatch):
    """The fused entry (affine + activation in the row kernels' store epilogue, residual as
    a pass) through every candidate plan (PO2Q_PLAN forces candidate i): tile, TT, loader
    wave and non-temporal-store variants alike."""
    N, C, H, W, K = shape
    torch.manual_seed(7)
    x = torch.randn(N, C, H, W, device=DEV)
    w = torch.randn(K, C, 3, 3, device=DEV) * 0.1
    ps = torch.rand(K, device=DEV) + 0.5
    pb = torch.randn(K, device=DEV) * 0.1
    res = torch.randn(N, K, H, W, device=DEV)
    base = _lib.qconv2d(x, w, None, 1, 1) * ps.view(1, -1, 1, 1) + pb.view(1, -1, 1, 1)
    n = len(_lib.plans(N, C, H, W, K, 3, 3, 1, 1))
    for i in range(n):
        monkeypatch.setenv("PO2Q_PLAN", str(i))
        for act, r in (("relu6", None), ("silu", res)):
            ref = base + (r if r is not None else 0)
            ref = torch.clamp(ref, 0, 6) if act == "relu6" else torch.nn.functional.silu(ref)
            y = _lib.qconv2d_fused(x, w, None, 1, 1, post_scale=ps, post_shift=pb, residual=r, act=act)
            err = ((y - ref).abs().max() / ref.abs().max()).item()
            assert err <= CONV_TOL, (i, act, err)


@pytest.mark.parametrize("shape", [(2, 64, 5, 56), (1, 64, 6, 40), (3, 64, 7, 8), (1, 64, 12, 36), (2, 64, 1, 60)],
                         ids=lambda s: "x".join(map(str, s)))
def test_c64_residual_in_kernel_every_plan_vs_oracle(shape, monkeypatch):
    """The BasicBlock conv2 of ResNet56 stage 3 (resnet.py:69-71: bn2(conv2(h)) + shortcut, ReLU)
    through the C = 64 row kernel's in-kernel residual (every candidate plan runs as its TT
    sibling with the residual ring; row counts cover every flush case of the 3-step unroll), against
    the oracle's fp64 conv of the bit-exact Q(w) with numpy affine / residual / ReLU."""
    N, C, H, W = shape
    g = torch.Generator().manual_seed(H * 100 + W)
    x = torch.randn(N, C, H, W, generator=g)
    w = torch.randn(C, C, 3, 3, generator=g) * 0.06
    ps = torch.rand(C, generator=g) + 0.5
    pb = torch.randn(C, generator=g) * 0.1
    res = torch.randn(N, C, H, W, generator=g)
    conv, _ = O.qconv2d(x.numpy(), w.numpy(), None, 1, 1, 1, 1, 4, "po2")
    ref = np.maximum(conv * ps.numpy().astype(np.float64).reshape(1, -1, 1, 1)
                     + pb.numpy().astype(np.float64).reshape(1, -1, 1, 1) + res.numpy().astype(np.float64), 0.0)
    xd, wd, psd, pbd, rd = (t.to(DEV) for t in (x, w, ps, pb, res))
    n = len(_lib.plans(N, C, H, W, C, 3, 3, 1, 1))
    for i in range(n):
        monkeypatch.setenv("PO2Q_PLAN", str(i))
        y = _lib.qconv2d_fused(xd, wd, None, 1, 1, post_scale=psd, post_shift=pbd, residual=rd, act="relu")
        err = normwise_err(y.cpu().numpy(), ref)
        assert err <= CONV_TOL, (i, _lib.plans(N, C, H, W, C, 3, 3, 1, 1)[i], err)


def test_c64_residual_in_kernel_full_size():
    """bs = 256 @56 (the BASELINE config's stage 3) with the in-kernel residual, against torch fp32."""
    torch.manual_seed(5)
    x = torch.relu(torch.randn(256, 64, 56, 56, device=DEV))
    w = torch.randn(64, 64, 3, 3, device=DEV) * 0.06
    ps = torch.rand(64, device=DEV) + 0.5
    pb = torch.randn(64, device=DEV) * 0.1
    res = torch.randn(256, 64, 56, 56, device=DEV)
    y = _lib.qconv2d_fused(x, w, None, 1, 1, post_scale=ps, post_shift=pb, residual=res, act="relu")
    ref = torch.relu(torch.nn.functional.conv2d(x, _lib.quantize(w, 4, "po2"), None, 1, 1) * ps.view(1, -1, 1, 1)
                     + pb.view(1, -1, 1, 1) + res)
    assert ((y - ref).abs().max() / ref.abs().max()).item() <= CONV_TOL


IMG_SHAPES = [(2, 16, 32, 32, 16), (2, 32, 16, 16, 32), (3, 64, 8, 8, 64), (1, 64, 7, 12, 64), (2, 32, 5, 8, 16),
              (2, 16, 9, 20, 32), (1, 64, 3, 4, 32), (2, 16, 1, 64, 64)]


@pytest.mark.parametrize("shape", IMG_SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_small_image_kernel_every_plan_vs_oracle(shape, monkeypatch):
    """The small-image kernel (po2q_conv_img.hip) through every one of its candidate plans (row
    segments, output-channel groups), plain and with the eval epilogue + residual, against the
    oracle's fp64 conv of the bit-exact Q(w): ragged row counts, groups spanning rows, K != C."""
    N, C, H, W, K = shape
    g = torch.Generator().manual_seed(N * 1000 + C * 10 + H)
    x = torch.randn(N, C, H, W, generator=g)
    w = torch.randn(K, C, 3, 3, generator=g) * 0.1
    ps = torch.rand(K, generator=g) + 0.5
    pb = torch.randn(K, generator=g) * 0.1
    res = torch.randn(N, K, H, W, generator=g)
    conv, _ = O.qconv2d(x.numpy(), w.numpy(), None, 1, 1, 1, 1, 4, "po2+")
    v = lambda t: t.numpy().astype(np.float64).reshape(1, -1, 1, 1)  # noqa: E731
    ref_epi = np.clip(conv * v(ps) + v(pb) + res.numpy().astype(np.float64), 0.0, 6.0)
    xd, wd, psd, pbd, rd = (t.to(DEV) for t in (x, w, ps, pb, res))
    plans = _lib.plans(N, C, H, W, K, 3, 3, 1, 1, mode="po2+")
    idx = [i for i, p in enumerate(plans) if "kind=bf16x3_img" in p]
    assert idx, plans
    for i in idx:
        monkeypatch.setenv("PO2Q_PLAN", str(i))
        y = _lib.qconv2d(xd, wd, None, 1, 1, 1, 1, 4, "po2+")
        err = normwise_err(y.cpu().numpy(), conv)
        assert err <= CONV_TOL, (plans[i], err)
        y = _lib.qconv2d_fused(xd, wd, None, 1, 1, 1, 1, 4, "po2+", post_scale=psd, post_shift=pbd, residual=rd,
                               act="relu6")
        err = normwise_err(y.cpu().numpy(), ref_epi)
        assert err <= CONV_TOL, (plans[i], "epilogue", err)


NONFINITE_SHAPES = [(2, 16, 12, 224, 16, 3, 1, 1), (2, 32, 10, 112, 32, 3, 1, 1), (2, 64, 9, 56, 64, 3, 1, 1),
                    (2, 16, 11, 64, 32, 3, 2, 1), (2, 32, 8, 32, 64, 1, 2, 0), (2, 24, 6, 6, 144, 1, 1, 0)]


def _nonfinite_input(N, C, H, W, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(N, C, H, W, generator=g)
    flat = x.view(-1)
    idx = torch.randperm(flat.numel(), generator=g)[:6]
    sig = torch.tensor([0x7F800001], dtype=torch.int32).view(torch.float32)  # signaling NaN, low payload only
    for v, i in zip((float("inf"), float("-inf"), float("nan"), float("inf"), sig.item(), float("-inf")), idx):
        flat[i] = v
    return x


def _same_nonfinite(y, ref):
    return (torch.equal(torch.isnan(y), torch.isnan(ref)) and torch.equal(torch.isposinf(y), torch.isposinf(ref))
            and torch.equal(torch.isneginf(y), torch.isneginf(ref)))


def _oracle_ref(x, w, st, pad, mode="po2"):
    """fp64 direct conv of Q(w) (the oracle): the mathematical non-finite pattern (a Winograd or
    FFT conv, as MIOpen may pick for torch's own conv, can turn +-inf into NaN)."""
    y, _ = O.qconv2d(x.cpu().numpy(), w.cpu().numpy(), None, st, pad, 1, 1, 4, mode)
    return torch.from_numpy(y).float()


@pytest.mark.parametrize("shape", NONFINITE_SHAPES, ids=[str(s) for s in NONFINITE_SHAPES])
def test_nonfinite_inputs_every_plan_match_oracle(shape):
    """+-inf and NaN activations (incl. a signaling NaN whose payload sits in the low 16 bits):
    every candidate plan reproduces the direct conv's NaN / +-inf pattern exactly (the bf16x3
    split clamps to +-FLT_MAX for mid / lo, hi keeps the non-finite value), finite outputs at
    the parity bar."""
    N, C, H, W, K, R, st, pad = shape
    x = _nonfinite_input(N, C, H, W, sum(shape)).to(DEV)
    g = torch.Generator().manual_seed(3)
    w = (torch.randn(K, C, R, R, generator=g) * 0.2).to(DEV)
    ref = _oracle_ref(x, w, st, pad)
    fin = torch.isfinite(ref)
    assert (~fin).any()
    bad = []
    for i, desc in enumerate(_lib.plans(N, C, H, W, K, R, R, st, pad)):
        y = _lib.qconv2d(x, w, None, st, pad, 1, 1, 4, "po2", plan=i).cpu()
        if not _same_nonfinite(y, ref):
            bad.append((i, desc.split(" tile")[0], int((torch.isnan(y) != torch.isnan(ref)).sum()),
                        int((torch.isinf(y) != torch.isinf(ref)).sum())))
            continue
        err = ((y[fin] - ref[fin]).abs().max() / ref[fin].abs().max()).item()
        assert err <= CONV_TOL, (desc, err)
    assert not bad, bad


@pytest.mark.parametrize("C,W", [(16, 224), (32, 112)])
def test_nonfinite_inputs_pair_and_s2ds(C, W):
    """The fused-block kernels keep the same non-finite pattern as the module sequence."""
    import torch.nn.functional as F

    x = _nonfinite_input(2, C, 10, W, C + W).to(DEV)
    g = torch.Generator().manual_seed(5)
    w1, w2 = (torch.randn(C, C, 3, 3, generator=g) * 0.1).to(DEV), (torch.randn(C, C, 3, 3, generator=g) * 0.1).to(DEV)
    y = _lib.qconv2d_pair(x, w1, w2, 4, "po2").cpu()
    h = _oracle_ref(x, w1, 1, 1)
    assert _same_nonfinite(y, _oracle_ref(h, w2, 1, 1))
    wd = (torch.randn(2 * C, C, 1, 1, generator=g) * 0.2).to(DEV)
    w3 = (torch.randn(2 * C, C, 3, 3, generator=g) * 0.1).to(DEV)
    y3, yd = _lib.qconv2d_s2ds(x, w3, wd, 4, "po2")
    assert _same_nonfinite(y3.cpu(), _oracle_ref(x, w3, 2, 1))
    assert _same_nonfinite(yd.cpu(), _oracle_ref(x, wd, 2, 0))


@pytest.mark.parametrize("N,H,W", [(2, 10, 112), (3, 30, 112), (1, 17, 112), (2, 112, 112)])
def test_s2ds_c32_segments_vs_oracle(N, H, W):
    """The C = 32 fused transition over ragged row segments: conv and shortcut outputs against the
    oracle, and the eval affine / ReLU epilogue equal to the same affine applied to the plain output."""
    C = 32
    g = torch.Generator().manual_seed(N * 7 + H + W)
    x = torch.randn(N, C, H, W, generator=g).to(DEV)
    w3 = (torch.randn(2 * C, C, 3, 3, generator=g) * 0.1).to(DEV)
    wd = (torch.randn(2 * C, C, 1, 1, generator=g) * 0.2).to(DEV)
    ps, pb = (torch.rand(2 * C, generator=g) + 0.5).to(DEV), (torch.randn(2 * C, generator=g) * 0.1).to(DEV)
    y3, yd = _lib.qconv2d_s2ds(x, w3, wd, 4, "po2")
    f3, fd = _lib.qconv2d_s2ds(x, w3, wd, 4, "po2", post_scale=ps, post_shift=pb, act="relu",
                               post_scale_ds=pb + 1.0, post_shift_ds=ps)
    aff = lambda t, a, b: t * a.view(1, -1, 1, 1) + b.view(1, -1, 1, 1)  # noqa: E731
    for f, r in ((f3, torch.relu(aff(y3, ps, pb))), (fd, aff(yd, pb + 1.0, ps))):
        assert ((f - r).abs().max() / r.abs().max()).item() <= CONV_TOL
    ref3, _ = O.qconv2d(x.cpu().numpy(), w3.cpu().numpy(), None, 2, 1, 1, 1, 4, "po2")
    refd, _ = O.qconv2d(x.cpu().numpy(), wd.cpu().numpy(), None, 2, 0, 1, 1, 4, "po2")
    assert normwise_err(y3.cpu().numpy(), ref3) <= CONV_TOL
    assert normwise_err(yd.cpu().numpy(), refd) <= CONV_TOL


PW_SHAPES = [  # N, C, HW side, K: MobileNetV2 @32 expand / project convs and odd edges
    (4, 16, 16, 96), (4, 96, 8, 24), (3, 24, 8, 144), (4, 144, 4, 32), (5, 160, 2, 960), (5, 960, 2, 160),
    (3, 32, 7, 64),   # HW = 49: 16-pixel groups span images, scalar stores
    (2, 8, 3, 12),    # C < 32, K < 16
    (7, 320, 1, 40),  # HW = 1
    (4, 960, 1, 160),  # HW = 1, C = 960: the split-K candidates
]


@pytest.mark.parametrize("shape", PW_SHAPES, ids=[str(s) for s in PW_SHAPES])
@pytest.mark.parametrize("mode", ["po2", "po2+"])
def test_pointwise_kernel_every_plan_vs_oracle(shape, mode):
    """The 1x1 GEMM kernel (kind bf16x3_pw: MobileNetV2 / MobileViT pointwise convs, reference
    models/mobilenet.py:78-93,120) is the planned kernel for every 1x1 / stride-1 shape, and every
    candidate plan meets the bar against the oracle, plain and with the fused BN + ReLU6 +
    residual epilogue (mobilenet.py:120-134)."""
    N, C, Hs, K = shape
    g = torch.Generator().manual_seed(N + C + K)
    x = torch.randn(N, C, Hs, Hs, generator=g)
    w = torch.randn(K, C, 1, 1, generator=g) * 0.2
    ps, pb = torch.rand(K, generator=g) + 0.5, torch.randn(K, generator=g) * 0.1
    res = torch.randn(N, K, Hs, Hs, generator=g)
    ref, _ = O.qconv2d(x.numpy(), w.numpy(), None, 1, 0, 1, 1, 4, mode)
    ref_e = np.clip(ref * ps.numpy().astype(np.float64).reshape(1, -1, 1, 1) +
                    pb.numpy().astype(np.float64).reshape(1, -1, 1, 1) + res.numpy().astype(np.float64), 0.0, 6.0)
    assert "kind=bf16x3_pw" in _lib.describe(N, C, Hs, Hs, K, 1, 1, 1, 0, 1, 1, 4, mode)
    xd, wd = x.to(DEV), w.to(DEV)
    plans = _lib.plans(N, C, Hs, Hs, K, 1, 1, 1, 0, 1, 1, 4, mode)
    assert sum("kind=bf16x3_pw" in d for d in plans) >= 1
    for i, desc in enumerate(plans):
        y = _lib.qconv2d(xd, wd, None, 1, 0, 1, 1, 4, mode, plan=i).cpu().numpy()
        assert normwise_err(y, ref) <= CONV_TOL, (desc, normwise_err(y, ref))
    y = _lib.qconv2d_fused(xd, wd, None, 1, 0, 1, 1, 4, mode, post_scale=ps.to(DEV), post_shift=pb.to(DEV),
                           residual=res.to(DEV), act="relu6").cpu().numpy()
    assert normwise_err(y, ref_e) <= CONV_TOL, normwise_err(y, ref_e)


def test_plain_conv_fused_stem_vs_torch():
    """The unquantized stems (resnet.py:99-102, mobilenet.py:41-46) as one native fp32 call with
    their eval BN + activation, against torch's fp32 module sequence."""
    from po2_quantization_amd.models.quantized_conv import plain_conv_fused

    torch.manual_seed(0)
    for cin, cout, k, st, act, mod in ((3, 16, 3, 1, "relu", torch.nn.ReLU()), (3, 32, 3, 2, "relu6", torch.nn.ReLU6()),
                                       (320, 1280, 1, 1, "relu6", torch.nn.ReLU6())):
        conv = torch.nn.Conv2d(cin, cout, k, st, k // 2, bias=False).to(DEV)
        bn = torch.nn.BatchNorm2d(cout).to(DEV).eval()
        with torch.no_grad():
            bn.running_mean.normal_(0, 0.1)
            bn.running_var.uniform_(0.5, 1.5)
            x = torch.randn(4, cin, 32 if k == 3 else 4, 32 if k == 3 else 4, device=DEV)
            y = plain_conv_fused(conv, x, bn=bn, act=act)
            ref = mod(bn(conv(x)))
        assert ((y - ref).abs().max() / ref.abs().max()).item() <= CONV_TOL


F32S_SHAPES = [  # N, C, H, W, K, R, stride, pad: unquantized stems and 1x1 convs (mode none)
    (2, 3, 32, 32, 16, 3, 1, 1), (2, 3, 33, 30, 32, 3, 2, 1), (3, 3, 15, 13, 16, 3, 2, 1), (2, 1, 9, 7, 20, 3, 1, 1),
    (2, 4, 10, 12, 24, 3, 1, 1), (4, 320, 2, 2, 1280, 1, 1, 0), (3, 96, 5, 5, 384, 1, 1, 0), (2, 30, 7, 7, 50, 1, 1, 0),
]


@pytest.mark.parametrize("shape", F32S_SHAPES, ids=[str(s) for s in F32S_SHAPES])
def test_unquantized_kernels_every_plan_vs_oracle(shape):
    """Mode "none" (the reference's plain nn.Conv2d stems / last 1x1 conv, and lin / lin+ weights):
    the direct fp32 stem kernel and the fp32-MFMA pointwise kernel, every candidate plan, plain and
    with the fused BN + ReLU6 epilogue, against the oracle's fp64 conv."""
    N, C, H, W, K, R, st, pad = shape
    g = torch.Generator().manual_seed(sum(shape))
    x = torch.randn(N, C, H, W, generator=g)
    w = torch.randn(K, C, R, R, generator=g) * 0.3
    b = torch.randn(K, generator=g) * 0.1
    ps, pb = torch.rand(K, generator=g) + 0.5, torch.randn(K, generator=g) * 0.1
    ref, _ = O.qconv2d(x.numpy(), w.numpy(), b.numpy(), st, pad, 1, 1, 4, "none")
    ref_e = np.clip(ref * ps.numpy().astype(np.float64).reshape(1, -1, 1, 1) +
                    pb.numpy().astype(np.float64).reshape(1, -1, 1, 1), 0.0, 6.0)
    desc0 = _lib.describe(N, C, H, W, K, R, R, st, pad, 1, 1, 4, "none")
    assert ("kind=direct_f32" in desc0) if R == 3 else ("kind=pw_f32" in desc0), desc0
    xd, wd, bd = x.to(DEV), w.to(DEV), b.to(DEV)
    for i, desc in enumerate(_lib.plans(N, C, H, W, K, R, R, st, pad, 1, 1, 4, "none")):
        y = _lib.qconv2d(xd, wd, bd, st, pad, 1, 1, 4, "none", plan=i).cpu().numpy()
        assert normwise_err(y, ref) <= CONV_TOL, (desc, normwise_err(y, ref))
    y = _lib.qconv2d_fused(xd, wd, bd, st, pad, 1, 1, 4, "none", post_scale=ps.to(DEV), post_shift=pb.to(DEV),
                           act="relu6").cpu().numpy()
    assert normwise_err(y, ref_e) <= CONV_TOL


@pytest.mark.parametrize("C,H,W", [(64, 56, 56), (64, 13, 44), (32, 20, 112), (16, 9, 224), (32, 7, 100)])
def test_fused_staging_plans_equal_packed_plans(C, H, W):
    """Every plan that quantizes + packs its weight inside the kernel (fp=1: the cooperative one-pass
    staging of po2q_quant_dev.h wq_pack_rows_lds / wq_pack_tap_row_lds) gives bit for bit the output of
    the same plan reading the separately packed weight (fp=0: pack_bf16x3_kernel), po2 and po2+."""
    g = torch.Generator().manual_seed(C * H + W)
    x = torch.randn(2, C, H, W, generator=g).to(DEV)
    w = (torch.randn(C, C, 3, 3, generator=g) * 0.1).to(DEV)
    for mode in ("po2", "po2+"):
        ds = _lib.plans(2, C, H, W, C, 3, 3, 1, 1, mode=mode)
        pairs = [(i, ds.index(d.replace(" fp=1", " fp=0"))) for i, d in enumerate(ds)
                 if " fp=1" in d and d.replace(" fp=1", " fp=0") in ds]
        assert pairs, (C, H, W, mode)
        for i, j in pairs:
            a = _lib.qconv2d(x, w, None, 1, 1, 1, 1, 4, mode, plan=i)
            b = _lib.qconv2d(x, w, None, 1, 1, 1, 1, 4, mode, plan=j)
            assert torch.equal(a, b), (C, H, W, mode, ds[i])
